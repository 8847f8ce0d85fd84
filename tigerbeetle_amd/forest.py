"""Host side of the forest's compaction schedule (restated for replays).

In a TigerBeetle replica the GPU path sits under Zig code that stays on the
host: `Forest.compact` -> `Groove.compact` -> `Tree.compact` decide, per
beat, which compactions start (src/lsm/tree.zig:612-712) from the Manifest's
levels (src/lsm/manifest.zig:470-574, manifest_level.zig:550-731), reserve
their blocks in the FreeSet (src/vsr/free_set.zig:225-345), and apply their
output tables to the Manifest at the half-bar end (tree.zig:876-976,
compaction.zig:936-985). To replay a workload through the engine (BASELINE
config 1: `tigerbeetle benchmark`'s load, benchmark_load.py) this module
restates that host logic; the compactions themselves run on an `executor`
(the GPU grid executor below, or the oracle in tests).

Blocks released by compactions (their input tables' data and index
blocks, compaction.zig:571-583) and by the manifest log's compaction
(manifest_log.zig:792) go to the FreeSet's staging and become free at the
next checkpoint (free_set.zig:383-390, 434-447), which the replica takes
after the bar of its trigger op (replica.zig:3470-3501, vsr.zig
Checkpoint: every vsr_checkpoint_interval ops). A restart from a checkpoint
(`Forest.restart`) restores the checkpointed manifest, free set and log,
forgets the grid's trusted blocks (a cold cache: every block is validated
before use), and replays the ops after the checkpoint with their memtable
puts while skipping the compactions the checkpoint already holds
(Tree.compact, tree.zig:627-646; superblock op_compacted).

Simplifications, stated in DESIGN.md §10: the blocks of the checkpoint's
own encoded free set and client replies are not simulated, so addresses
differ from a replica's by those blocks; every address a compaction uses is
still a FreeSet acquire from its own reservation.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

import numpy as np

from . import trees
from .tables import EVENT_INSERT, EVENT_REMOVE, EVENT_UPDATE, SNAPSHOT_LATEST, TableInfo

LSM_LEVELS = trees.LSM_LEVELS            # config.zig:140
GROWTH = trees.LSM_GROWTH_FACTOR         # config.zig:141
BAR = trees.LSM_BATCH_MULTIPLE           # config.zig:142
HALF = BAR // 2
# constants.zig:47-49 with the production config (config.zig:133-142): 1024
# journal slots - 32 - 32 * ceil(8 / 32) = 960 ops between checkpoints.
VSR_CHECKPOINT_INTERVAL = 1024 - BAR - BAR * -(-8 // BAR)


def checkpoint_after(checkpoint: int, interval: int = VSR_CHECKPOINT_INTERVAL) -> int:
    """vsr.Checkpoint.checkpoint_after (vsr.zig:1343-1361)."""
    return interval - 1 if checkpoint == 0 else checkpoint + interval


def trigger_for_checkpoint(checkpoint: int) -> int:
    """vsr.Checkpoint.trigger_for_checkpoint (vsr.zig:1364-1371): the op whose
    compaction completes the checkpoint's bar."""
    return checkpoint + BAR


def table_count_max_for_level(level: int) -> int:
    """tree.zig:1114-1119."""
    return GROWTH ** (level + 1)


def compaction_op_min(op: int) -> int:
    """tree.zig:1093-1095."""
    return op - op % HALF


def snapshot_min_for_table_output(op_min: int) -> int:
    """compaction.zig:981-985."""
    return op_min + HALF


def snapshot_max_for_table_input(op_min: int) -> int:
    """compaction.zig:977-979."""
    return snapshot_min_for_table_output(op_min) - 1


class FreeSet:
    """FreeSet.reserve/acquire/forfeit (free_set.zig:225-345) over a bitmap."""

    def __init__(self, block_count: int):
        self.acquired = np.zeros(block_count, dtype=bool)
        self.staging = np.zeros(block_count, dtype=bool)  # released, free at the next checkpoint
        self.reservation_blocks = 0
        self.reservation_count = 0
        self.released = 0
        self.reused = 0  # acquires of addresses freed by a checkpoint

    def reserve(self, count: int) -> tuple:
        base = self.reservation_blocks
        free = np.flatnonzero(~self.acquired[base:])
        if len(free) < count:
            raise RuntimeError("grid full: raise the replay's block count")
        end = base + int(free[count - 1]) + 1
        self.reservation_blocks = end
        self.reservation_count += 1
        return (base, end - base)

    def addresses(self, reservation: tuple) -> np.ndarray:
        """The acquire() sequence of a reservation: its free blocks in order."""
        base, count = reservation
        return (np.flatnonzero(~self.acquired[base:base + count]) + base + 1).astype(np.uint64)

    def acquire(self, addresses) -> None:
        a = np.asarray(addresses, dtype=np.int64)
        assert not self.acquired[a - 1].any()
        self.acquired[a - 1] = True
        if self.freed is not None:
            self.reused += int(self.freed[a - 1].sum())

    freed = None  # blocks a checkpoint freed (statistics: reuse)

    def acquire_from(self, reservation: tuple) -> int:
        """FreeSet.acquire(reservation) (free_set.zig:280-311): the first free
        block of the reservation, now acquired (the manifest log's blocks)."""
        base, count = reservation
        free = np.flatnonzero(~self.acquired[base:base + count])
        assert len(free), "reservation exhausted"
        address = base + int(free[0]) + 1
        self.acquired[address - 1] = True
        return address

    def release(self, address: int) -> None:
        """FreeSet.release (free_set.zig:383-390): staged until the next
        checkpoint; still acquired until then (no reservation may reuse it)."""
        assert self.acquired[address - 1] and not self.staging[address - 1]
        self.staging[address - 1] = True
        self.released += 1

    def checkpoint(self) -> int:
        """FreeSet.checkpoint (free_set.zig:434-447): every staged block is
        freed; no reservation may be outstanding. Returns the count."""
        assert self.reservation_count == 0 and self.reservation_blocks == 0
        n = int(self.staging.sum())
        self.freed = self.staging.copy() if self.freed is None else (self.freed | self.staging)
        self.acquired &= ~self.staging
        self.staging[:] = False
        return n

    def snapshot(self) -> dict:
        assert self.reservation_count == 0
        return {"acquired": self.acquired.copy(), "staging": self.staging.copy()}

    def restore(self, snap: dict) -> None:
        self.acquired, self.staging = snap["acquired"].copy(), snap["staging"].copy()
        self.reservation_blocks = self.reservation_count = 0

    def forfeit(self) -> None:
        self.reservation_count -= 1
        if self.reservation_count == 0:
            self.reservation_blocks = 0


class Level:
    """ManifestLevel: tables ordered by (key_max, snapshot_min)
    (manifest_level.zig:41-70); invisible tables stay until
    remove_invisible removes them."""

    def __init__(self):
        self.tables: list = []

    def visible(self) -> list:
        return [t for t in self.tables if t.snapshot_max == SNAPSHOT_LATEST]

    def insert(self, t: TableInfo) -> None:
        self.tables.append(t)
        self.tables.sort(key=lambda x: (x.key_max, x.snapshot_min))

    def set_snapshot_max(self, t: TableInfo, snapshot: int) -> TableInfo:
        """ManifestLevel.set_snapshot_max (manifest_level.zig:243-266)."""
        assert t.snapshot_max == SNAPSHOT_LATEST and snapshot < SNAPSHOT_LATEST - 1
        u = replace(t, snapshot_max=snapshot)
        self.tables[self.tables.index(t)] = u
        return u

    def remove_invisible(self, key_min: int, key_max: int) -> list:
        """The tables Manifest.remove_invisible_tables removes, in its order
        (manifest.zig:345-386 over ManifestLevel.iterator(.invisible, &.{},
        .descending, range), manifest_level.zig:327-520): start at the last
        table sharing the key_max of the first table whose key_max >= the
        range's key_max (or at the last table), walk down; skip visible tables
        and tables starting above the range; stop at the first invisible table
        ending below it."""
        n = len(self.tables)
        if n == 0:
            return []
        kmax = [t.key_max for t in self.tables]
        lb = next((i for i, k in enumerate(kmax) if k >= key_max), n)
        if lb == n:
            start = n - 1
        else:
            start = lb
            while start + 1 < n and kmax[start + 1] == kmax[lb]:
                start += 1
        removed = []
        for i in range(start, -1, -1):
            t = self.tables[i]
            if t.snapshot_max == SNAPSHOT_LATEST:
                continue
            if t.key_min > key_max:
                continue
            if t.key_max < key_min:
                break
            removed.append(t)
        for t in removed:
            self.tables.remove(t)
        return removed

    def overlapping(self, key_min: int, key_max: int, max_tables: int):
        """tables_overlapping_with_key_range (manifest_level.zig:677-731)."""
        kmin, kmax, found = key_min, key_max, []
        for t in self.visible():
            if t.key_max < key_min or t.key_min > key_max:
                continue
            kmin, kmax = min(kmin, t.key_min), max(kmax, t.key_max)
            if len(found) == max_tables:
                return None
            found.append(t)
        return (kmin, kmax, found)


@dataclass
class Compaction:
    """One started Compaction (compaction.zig:84-99, 280-404)."""
    tree: trees.TreeSpec
    level_b: int
    op_min: int
    table_a: TableInfo | None           # None: the immutable table
    range_b: tuple                      # (key_min, key_max, [TableInfo])
    drop_tombstones: bool
    move: bool
    reservation: tuple | None = None
    addresses: np.ndarray | None = None
    outputs: list = field(default_factory=list)  # TableInfos (after the batch)
    result: object = None

    @property
    def snapshot_min(self) -> int:
        return snapshot_min_for_table_output(self.op_min)


class Tree:
    """One LSM tree's host state: mutable/immutable table bookkeeping, the
    manifest's levels and the per-half-bar compactions."""

    def __init__(self, spec: trees.TreeSpec):
        self.spec = spec
        self.levels = [Level() for _ in range(LSM_LEVELS)]
        self.mutable_count = 0
        self.mutable_keys = [None, None]      # (min, max) of the mutable table's keys
        self.mutable_sorted = True            # puts arrived in key order (table_memory.zig:83-87)
        self.immutable_count = 0
        self.immutable_keys = [None, None]
        self.immutable_sorted = True
        self.immutable_flushed = True
        self.compactions: list = []

    # -- TableMemory ------------------------------------------------------
    def put_keys(self, n: int, key_min: int, key_max: int, in_order: bool = True, first: int | None = None) -> None:
        """TableMemory.put of a batch: count, key range, and whether the
        table is still sorted (the batch in order and not below the last key)."""
        if self.mutable_keys[1] is not None and (not in_order or (first if first is not None else key_min) <
                                                 self.mutable_keys[1]):
            self.mutable_sorted = False
        if not in_order:
            self.mutable_sorted = False
        self.mutable_count += n
        lo, hi = self.mutable_keys
        self.mutable_keys = [key_min if lo is None else min(lo, key_min), key_max if hi is None else max(hi, key_max)]
        assert self.mutable_count <= self.spec.value_count_max

    def swap_mutable_and_immutable(self) -> bool:
        """tree.zig:979-999; returns whether the new immutable table has values."""
        assert self.immutable_flushed
        self.immutable_count, self.immutable_keys = self.mutable_count, self.mutable_keys
        self.immutable_sorted = self.mutable_sorted
        self.immutable_flushed = self.immutable_count == 0
        self.mutable_count, self.mutable_keys, self.mutable_sorted = 0, [None, None], True
        return self.immutable_count > 0

    # -- Manifest ---------------------------------------------------------
    def must_drop_tombstones(self, level_b: int, rng: tuple) -> bool:
        """manifest.zig:547-574."""
        for level_c in range(level_b + 1, LSM_LEVELS):
            if self.levels[level_c].overlapping(rng[0], rng[1], 1 << 30)[2]:
                return False
        return True

    def compaction_table(self, level_a: int):
        """manifest.zig:484-512 + manifest_level.zig:550-594."""
        la, lb = self.levels[level_a], self.levels[level_a + 1]
        if len(la.visible()) < table_count_max_for_level(level_a):
            return None
        best = None
        for t in la.visible():
            r = lb.overlapping(t.key_min, t.key_max, GROWTH)
            if r is None:
                continue
            if best is None or len(r[2]) < len(best[1][2]):
                best = (t, r)
            if not best[1][2]:
                break
        assert best is not None
        return best

    def start_half_bar(self, op: int, free_set: FreeSet) -> list:
        """Tree.compact at a half-bar start (tree.zig:661-690): the immutable
        table's compaction (odd half), then one per level pair."""
        beat = op % BAR
        odd = beat == HALF
        op_min = compaction_op_min(op)
        started = []
        if odd and not self.immutable_flushed:
            r = self.levels[0].overlapping(self.immutable_keys[0], self.immutable_keys[1], GROWTH)
            assert r is not None
            started.append(Compaction(self.spec, 0, op_min, None, r, self.must_drop_tombstones(0, r), False))
        for level_a in range(1 if odd else 0, LSM_LEVELS - 1, 2):
            sel = self.compaction_table(level_a)
            if sel is None:
                continue
            t, r = sel
            move = not r[2]
            started.append(Compaction(self.spec, level_a + 1, op_min, t, r,
                                      self.must_drop_tombstones(level_a + 1, r), move))
        block_count_max = self.spec.layout()["block_count_max"]
        for c in started:
            if not c.move:  # compaction.zig:300-318
                c.reservation = free_set.reserve((len(c.range_b[2]) + 1) * block_count_max)
                c.addresses = free_set.addresses(c.reservation)
        self.compactions = started
        return started

    def apply(self, c: Compaction, log=None) -> None:
        """Compaction.apply_to_manifest (compaction.zig:939-973) then the
        remove_invisible_tables calls of Tree.compact_end (tree.zig:905-953),
        appending each event to the manifest log `log` (manifest.zig:233-386):
        updates of the inputs (A at level_b - 1, then every B table), inserts
        of the outputs or the move's update at level_b, removes of the inputs."""
        snap_max = snapshot_max_for_table_input(c.op_min)
        lb = self.levels[c.level_b]
        tid, ks = self.spec.tree_id, self.spec.key_size

        def emit(t: TableInfo, level: int, event: int) -> None:
            if log is not None:
                log.append(t.encode(tid, level, event, ks))

        if c.move:
            la = self.levels[c.level_b - 1]
            la.tables.remove(c.table_a)               # no remove event (manifest.zig:301-308)
            moved = replace(c.table_a, level=c.level_b)
            lb.insert(moved)
            emit(moved, c.level_b, EVENT_UPDATE)
        else:
            if c.table_a is not None:
                emit(self.levels[c.level_b - 1].set_snapshot_max(c.table_a, snap_max), c.level_b - 1, EVENT_UPDATE)
            for t in c.range_b[2]:
                emit(lb.set_snapshot_max(t, snap_max), c.level_b, EVENT_UPDATE)
            for t in c.outputs:
                lb.insert(t)
                emit(t, c.level_b, EVENT_INSERT)
        kmin, kmax = c.range_b[0], c.range_b[1]
        levels = [c.level_b] if c.table_a is None else [c.level_b] + ([c.level_b - 1] if c.level_b > 0 else [])
        for level in levels:
            for t in self.levels[level].remove_invisible(kmin, kmax):
                emit(t, level, EVENT_REMOVE)


class Forest:
    """Forest.compact over the trees a workload touches, in the forest's
    order (grooves accounts, transfers; per groove: ids, objects, indexes:
    forest.zig:319-342, groove.zig:1084-1104)."""

    ORDER = ["accounts.id", "accounts.timestamp", "accounts.user_data_128", "accounts.user_data_64",
             "accounts.user_data_32", "accounts.ledger", "accounts.code",
             "transfers.id", "transfers.timestamp", "transfers.debit_account_id", "transfers.credit_account_id",
             "transfers.amount", "transfers.pending_id", "transfers.user_data_128", "transfers.user_data_64",
             "transfers.user_data_32", "transfers.timeout", "transfers.ledger", "transfers.code"]

    def __init__(self, executor, block_count: int, cluster: int = 0, manifest_log: bool = True,
                 block_size: int = 1 << 20, checkpoint_interval: int | None = VSR_CHECKPOINT_INTERVAL):
        from .manifest import ManifestLog
        self.executor = executor
        self.block_size = block_size
        self.free_set = FreeSet(block_count)
        # Checkpoints (replica.zig:3470-3501): after the bar of each trigger op.
        self.checkpoint_interval = checkpoint_interval
        self.op_checkpoint = 0
        self.checkpoints: list = []       # (checkpoint op, trigger op, blocks freed)
        self._snapshot = None             # host state at the last checkpoint (restart)
        self.op_compacted_max = 0         # after a restart: ops <= this skip compaction (op_compacted)
        self.table_blocks: dict = {}      # index block address -> the table's block addresses
        self.trees = {name: Tree(trees.BY_NAME[name]) for name in self.ORDER}
        self.cluster = cluster
        self.pending = None       # (batch handle, [Compaction]) of the running half-bar
        self.history: list = []   # per half-bar: (op, [Compaction]) once applied
        self.swaps: list = []     # per bar end: [(tree, values, sorted)] made immutable
        # The forest's manifest log (forest.zig:197-204), its blocks closed by
        # the executor's store (the GPU grid, or the oracle in tests).
        self.manifest_log = ManifestLog(executor.manifest_store(cluster), self.free_set, block_size) \
            if manifest_log and hasattr(executor, "manifest_store") else None

    def put(self, name: str, values: np.ndarray) -> None:
        spec = self.trees[name].spec
        first, key_min, key_max, in_order = key_summary(values, spec)
        self.trees[name].put_keys(len(values), key_min, key_max, in_order, first)
        self.executor.put(name, values)

    def compact(self, op: int) -> None:
        """Forest.compact(op) (forest.zig:319-342) then compact_end."""
        beat = op % BAR
        skipped = op <= self.op_compacted_max  # recovered: the checkpoint holds this op's compaction
        if op >= BAR and beat in (0, HALF):
            started = []
            for name in self.ORDER:
                if skipped:
                    self.trees[name].compactions = []
                    continue
                for c in self.trees[name].start_half_bar(op, self.free_set):
                    started.append((name, c))
            if self.manifest_log is not None:  # after the grooves (forest.zig:323-331)
                self.manifest_log.compact(op, skipped=skipped)
            jobs = [(name, c) for name, c in started if not c.move]
            handle = self.executor.submit(jobs, self.cluster) if jobs else None
            self.pending = (handle, started)
        if op >= BAR and beat in (HALF - 1, BAR - 1):
            handle, started = self.pending
            if handle is not None:
                self.executor.wait(handle, [c for _, c in started if not c.move])
            odd = beat == BAR - 1
            for name, c in started:  # the blocks each compaction wrote
                if not c.move:
                    self.free_set.acquire(c.addresses[:c.result.block_count])
                    self.record_blocks(c)
            # Grooves' compact_end in forest order, each tree's immutable
            # compaction first, then its level compactions (tree.zig:876-953).
            log = self.manifest_log
            for name in self.ORDER:
                mine = [c for n, c in started if n == name]
                for c in mine:
                    if c.table_a is None:
                        self.trees[name].apply(c, log)
                        self.trees[name].immutable_flushed = True
                        self.executor.flushed(name)
                for c in mine:
                    if c.table_a is not None:
                        self.trees[name].apply(c, log)
            for name, c in started:
                if not c.move:
                    self.free_set.forfeit()
            if log is not None and beat in (HALF - 1, BAR - 1):
                log.compact_end()
            assert odd or not any(c.table_a is None for _, c in started)
            self.history.append((op, started))
            self.pending = None
        if beat == BAR - 1:
            swapped = [name for name in self.ORDER if self.trees[name].swap_mutable_and_immutable()]
            self.swaps.append([(name, self.trees[name].immutable_count, self.trees[name].immutable_sorted)
                               for name in swapped])
            # TableMemory.sort skips a table whose puts arrived in key order
            # (table_memory.zig:110-150): only the others are sorted.
            self.executor.swap([name for name in swapped if not self.trees[name].immutable_sorted])
            if self.checkpoint_interval and op == trigger_for_checkpoint(
                    checkpoint_after(self.op_checkpoint, self.checkpoint_interval)):
                self.checkpoint(checkpoint_after(self.op_checkpoint, self.checkpoint_interval), op)

    def record_blocks(self, c: Compaction) -> None:
        """The output tables' blocks (data blocks then the index block per
        table, in acquire order: compaction.zig:806-886), and the input
        tables' blocks released (release_table_blocks, compaction.zig:571-583:
        staged until the next checkpoint)."""
        dbcm = c.tree.layout(self.block_size)["data_block_count_max"]
        db = c.result.data_block_count
        for t, info in enumerate(c.outputs):
            k0, k_last = t * dbcm, min((t + 1) * dbcm, db) - 1
            slots = [k + k // dbcm for k in range(k0, k_last + 1)] + [k_last + t + 1]
            blocks = [int(c.addresses[s]) for s in slots]
            assert blocks[-1] == info.address
            self.table_blocks[info.address] = blocks
        for t in ([c.table_a] if c.table_a is not None else []) + list(c.range_b[2]):
            for address in self.table_blocks.pop(t.address):
                self.free_set.release(address)

    def checkpoint(self, op_checkpoint: int, trigger: int) -> None:
        """The replica's checkpoint after its trigger op's bar (replica.zig
        commit_op_compact_callback -> checkpoint_data; forest.zig:422-445):
        the manifest log closes its partial block (manifest_log.zig:767-781),
        the free set frees every staged block (free_set.zig:434-447), and the
        host state is what a restart recovers."""
        if self.manifest_log is not None:
            self.manifest_log.checkpoint()
        freed = self.free_set.checkpoint()
        if hasattr(self.executor, "checkpoint"):
            self.executor.checkpoint()
        self.op_checkpoint = op_checkpoint
        self.checkpoints.append((op_checkpoint, trigger, freed))
        self._snapshot = self.snapshot()

    def snapshot(self) -> dict:
        """What the checkpoint persists: the manifest (every tree's levels),
        the free set, the manifest log, the tables' block lists."""
        import copy
        log = self.manifest_log
        return {
            "levels": {name: copy.deepcopy(t.levels) for name, t in self.trees.items()},
            "free_set": self.free_set.snapshot(),
            "log": None if log is None else log.snapshot(),
            "table_blocks": {a: list(b) for a, b in self.table_blocks.items()},
            "op_checkpoint": self.op_checkpoint,
        }

    def restart(self) -> int:
        """Crash and recover from the last checkpoint (replica open ->
        superblock, manifest log open, free set decode): the host state is the
        checkpoint's, memtables are empty, the grid's cache is cold (the
        executor forgets every trusted block), and the ops after the
        checkpoint are replayed with their compactions skipped up to the
        trigger op (tree.zig:627-646). Returns the first op to replay."""
        import copy
        snap = self._snapshot
        assert snap is not None, "no checkpoint to restart from"
        for name, t in self.trees.items():
            fresh = Tree(t.spec)
            fresh.levels = copy.deepcopy(snap["levels"][name])
            self.trees[name] = fresh
        self.free_set.restore(snap["free_set"])
        if self.manifest_log is not None:
            self.manifest_log.restore(snap["log"])
        self.table_blocks = {a: list(b) for a, b in snap["table_blocks"].items()}
        self.op_checkpoint = snap["op_checkpoint"]
        self.op_compacted_max = trigger_for_checkpoint(self.op_checkpoint)
        self.pending = None
        if hasattr(self.executor, "restart"):
            self.executor.restart()
        return self.op_checkpoint + 1

    def checkpoint_manifest(self) -> None:
        """ManifestLog.checkpoint (manifest_log.zig:767-781) at the end of a
        replay: the partial block is closed, so every event is in a block."""
        if self.manifest_log is not None:
            self.manifest_log.checkpoint()

    def run(self, load_ops, progress=None, start: int = 1, stop: int | None = None) -> None:
        """Commit every op of a workload: its puts, then Forest.compact(op);
        ops before `start` (already committed: a restart replays from the
        checkpoint) and after `stop` (a crash) are not committed."""
        for op in load_ops:
            if op.op < start:
                continue
            if stop is not None and op.op > stop:
                break
            for name, values in op.puts.items():
                self.put(name, values)
            self.compact(op.op)
            if progress:
                progress(op.op)


def unique_keys(name: str) -> bool:
    """Trees whose keys are never put twice in the benchmark's state machine
    (TBC_COMPACTION_UNIQUE_KEYS): transfers are immutable (every transfer
    tree's key holds the transfer's unique timestamp or id), and an account's
    id and indexed fields never change after creation (state_machine.zig
    create_account; balance updates re-put only the accounts object tree,
    groove.zig:911-1006). The engine verifies it on the device and recomputes
    a compaction whose speculation breaks."""
    return name != "accounts.timestamp"


def key_summary(values: np.ndarray, spec: trees.TreeSpec) -> tuple:
    """(first key, min key, max key, keys non-decreasing) of a put batch,
    keys as integers (key_from_value: composite_key.zig:48-50, groove.zig)."""
    from . import workloads
    limbs = workloads.keys_of(values, spec)  # least significant limb first

    def extreme(pick):
        idx = np.arange(len(limbs[0]))
        for l in reversed(limbs):  # most significant limb first
            v = l[idx]
            idx = idx[v == pick(v)]
        return sum(int(l[idx[0]]) << (64 * i) for i, l in enumerate(limbs))

    # consecutive keys in order: compare limbs from the most significant one
    decided = np.zeros(max(0, len(limbs[0]) - 1), dtype=bool)
    ok = np.ones_like(decided)
    for l in reversed(limbs):
        lt, gt = l[:-1] < l[1:], l[:-1] > l[1:]
        ok &= ~(gt & ~decided)
        decided |= lt | gt
    first = sum(int(l[0]) << (64 * i) for i, l in enumerate(limbs))
    return first, extreme(np.min), extreme(np.max), bool(ok.all())


class GridExecutor:
    """Runs a Forest's compactions on the GPU: memtables on the device
    (tbc_memtable), the bar-end sorts as one segmented batch, each half-bar's
    compactions as one batch over the GPU-resident grid."""

    def __init__(self, engine, grid, record: bool = False):
        from .engine import Memtable
        self.engine, self.grid = engine, grid
        self._Memtable = Memtable
        self.mutable, self.immutable = {}, {}
        # record=True keeps every GPU work item and a device copy of each
        # memtable as it was before its sort, so that the whole replay can be
        # re-executed with its inputs resident in HBM (bench.py --config 1).
        self.recording = record
        self.record: list = []
        self.frozen: dict = {}  # recording: name -> (device copy, count) of an unsorted immutable table
        self.archive: list = []
        self.puts_bytes = 0

    def manifest_store(self, cluster: int):
        from .manifest import GridManifestStore
        return GridManifestStore(self.grid, cluster, self.record if self.recording else None)

    def _mem(self, name: str):
        if name not in self.mutable:
            spec = trees.BY_NAME[name]
            self.mutable[name] = self._Memtable(self.engine, spec)
            self.immutable[name] = self._Memtable(self.engine, spec)
        return self.mutable[name]

    def put(self, name: str, values: np.ndarray) -> None:
        self._mem(name).put(values)
        self.puts_bytes += values.nbytes

    def swap(self, names: list) -> None:
        """Bar end: every mutable table becomes immutable (its immutable table
        was flushed by the bar's first half); the ones named are sorted, by
        one out-of-place sort into the immutable tables' buffers
        (tbc_memtable_make_immutable), the others trade buffers."""
        sort = set(names)
        pairs = []
        for name in list(self.mutable):
            self.immutable[name].reset()  # make_mutable after its flush
            pairs.append((name, self.mutable[name], self.immutable[name]))
        # Recording: each table as put is copied first, so that a replay of
        # the record sorts it again from that copy (straight into the
        # immutable buffer, as here), and a table that needs no sort is
        # compacted from its copy (the buffer holds a later bar by then).
        archived = {}
        if self.recording:
            for name, m, _ in pairs:
                ptr, n = m.values()
                if n == 0:
                    continue
                nbytes = n * trees.BY_NAME[name].value_size
                copy = self.engine.alloc(nbytes)
                self.engine.copy_device_async(copy.ptr, ptr, nbytes)
                self.archive.append(copy)
                archived[name] = (copy.ptr, n)
        self._Memtable.make_immutable(self.engine, [(m, im, name not in sort) for name, m, im in pairs])
        self.frozen = {}
        if self.recording:
            jobs = []
            for name, _, im in pairs:
                if name not in archived:
                    continue
                if name in sort:
                    out, n = im.values()
                    jobs.append((trees.BY_NAME[name], archived[name][0], n, out))
                else:
                    self.frozen[name] = archived[name]
            if jobs:
                self.record.append(("sort", jobs))

    def flushed(self, name: str) -> None:
        pass  # the immutable memtable is reset when it becomes mutable again (swap)

    def checkpoint(self) -> None:
        """The replica checkpoints with no grid IO in flight
        (grid.assert_only_repairing): a replay of the record waits here."""
        if self.recording:
            self.record.append(("checkpoint",))

    def restart(self) -> None:
        """A restart: memtables empty, the grid's cache cold."""
        for name in list(self.mutable):
            self.mutable[name].reset()
            self.immutable[name].reset()
        self.frozen = {}
        self.grid.invalidate()
        if self.recording:
            self.record.append(("restart",))

    def submit(self, jobs: list, cluster: int):
        from . import abi
        from .engine import Job
        js = []
        for name, c in jobs:
            if c.table_a is None:
                ptr, n = self.frozen.get(name) or self.immutable[name].values()
                segs_a, tables_a = [(ptr, n)], []
            else:
                segs_a, tables_a = [], [c.table_a.ref()]
            flags = abi.COMPACTION_GRID | (abi.COMPACTION_UNIQUE_KEYS if unique_keys(name) else 0)
            js.append(Job(c.tree, segs_a, [], c.table_a is None, c.drop_tombstones, c.level_b, cluster,
                          c.snapshot_min, c.addresses, None, flags=flags, grid=self.grid,
                          tables_a=tables_a, tables_b=[t.ref() for t in c.range_b[2]]))
        if self.recording:
            self.record.append(("batch", js))
        return self.engine.submit(js)

    def wait(self, handle, compactions: list) -> None:
        handle.wait()
        for i, c in enumerate(compactions):
            r, infos = handle.result(i)
            if r.status != 0:  # a block error or invariant is never applied to the manifest
                from .abi import TbcError
                raise TbcError(r.status, f"compaction {i} ({c.tree.name}, level_b {c.level_b})")
            c.result = r
            c.outputs = [TableInfo.decode(raw, c.tree.key_size) for raw in infos]
        handle.release()
