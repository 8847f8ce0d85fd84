"""Key-range split of ONE compaction across ranks.

A half-bar's compactions shard by job (shard.py). A single job can also be
split across GPUs by key range: equal keys never straddle a splitter, so every
rank's sub-compaction decides exactly the survivors the whole job would
(dedup of immutable runs, secondary-index cancellation and tombstone dropping
are per key: compaction.zig:483-559, 647-804). What a rank cannot know alone is
WHERE its survivors fall in the job's output: data blocks are cut every
`block_value_count_max` survivors and tables every `data_block_count_max`
blocks (compaction.zig:806-886), counted from the job's first survivor. So:

1. Splitters: P-1 keys, and the cuts (lower bounds of each splitter in A
   and in B), identical on every rank without communication. Two ways:
   `block_splitters` + `block_cuts` (what a rank on a node uses): the
   splitters are data-block first keys (TableIndex.keys_min of the input
   tables' index blocks, schema.zig:80-260) balanced by the blocks' value
   counts, and each cut is a lower bound inside the one data block of A and
   of each B table that can hold it, so a rank reads the index keys plus at
   most two data blocks per input table, and stages only the blocks of its
   own range (`rank_blocks`); or `split_points`, exact merge-path
   co-ranking over A ∪ B, for a caller that holds every key anyway.
2. Counts: each rank merges its key range without writing anything
   (TBC_COMPACTION_COUNT_ONLY) for its survivor count c_p; an all-gather of
   the counts and an exclusive scan give every rank its global output
   offset o_p (`plan_split`).
3. Bodies in place: each rank merges its range again (VALUES_ONLY with
   tbc_compaction.output_offset = o_p), writing every survivor at its global
   output position: its data block and slot in the job's own block layout.
4. Data block k belongs to the rank holding its first value (k·vcm); the
   values of a block that starts on an earlier rank (at most one block per
   rank: positions [o_p, first block boundary)) go to that block's owner
   (all-gather of ≤ vcm - 1 values per rank, one copy on the owner).
5. Each rank finishes the data blocks it owns in place (tbc_compaction_seal:
   AEGIS-128L body and header checksums, data_block_finish) and writes their
   index entries (checksum, key_min, key_max, address) into their tables'
   index block slots.
6. Table t belongs to the owner of its first data block. A rank whose first
   block is inside an earlier rank's table sends that table's owner its
   entries (all-gather of ≤ dbcm - 1 entries per rank, 40 + 2·key_size
   bytes each); the owner copies them into its index block image and seals
   its tables (index_block_finish, TableInfo).

No value moves twice: the rank merges write the bodies where the blocks
are, and only one partial block's values plus one table's index entries per
rank cross ranks. The blocks, checksums and TableInfos are the unsplit job's
byte for byte (the union over ranks of each rank's data blocks
`plan.blocks(p)` and tables `plan.tables(p)`; tested against the oracle).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .abi import COMPACTION_VALUES_ONLY as VALUES_ONLY

HEADER_SIZE = 256


# ---------------------------------------------------------------------------
# Splitters (host: keys of the job's inputs, most significant limb last).

def _key(limbs: list, i: int) -> tuple:
    return tuple(int(l[i]) for l in reversed(limbs))


def lower_bound(limbs: list, n: int, key: tuple) -> int:
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if _key(limbs, mid) < key:
            lo = mid + 1
        else:
            hi = mid
    return lo


def split_points(a_limbs: list, na: int, b_limbs: list, nb: int, world: int) -> list:
    """[(a_cut, b_cut)] * (world + 1): rank p takes A[a_cut[p]:a_cut[p+1]] and
    B[b_cut[p]:b_cut[p+1]]. The split of rank p sits at merged position
    p·(na+nb)/world (merge path, A before B on equal keys), moved back to the
    first position of that key so that no key straddles two ranks."""
    assert world >= 1
    cuts = [(0, 0)]
    for p in range(1, world):
        t = p * (na + nb) // world
        lo, hi = max(0, t - nb), min(t, na)
        while lo < hi:  # smallest i with not (A[i] <= B[t-i-1])
            i = (lo + hi) // 2
            if _key(a_limbs, i) <= _key(b_limbs, t - i - 1):
                lo = i + 1
            else:
                hi = i
        i, j = lo, t - lo
        cand = ([_key(a_limbs, i)] if i < na else []) + ([_key(b_limbs, j)] if j < nb else [])
        if not cand:
            cuts.append((na, nb))
            continue
        s = min(cand)
        a_cut, b_cut = lower_bound(a_limbs, na, s), lower_bound(b_limbs, nb, s)
        pa, pb = cuts[-1]
        cuts.append((max(a_cut, pa), max(b_cut, pb)))
    cuts.append((na, nb))
    return cuts


class BlockedSide:
    """One input side (A, or B's tables concatenated) as its data blocks:
    `first_keys[j]` = the key of block j's first value (from the index
    block), `counts[j]` its values, and `keys(j)` the limb arrays of block j
    (read on demand: only boundary blocks are ever asked for)."""

    def __init__(self, first_keys: list, counts: list, keys):
        self.first_keys, self.counts, self.keys = first_keys, [int(c) for c in counts], keys
        self.starts = [0]
        for c in self.counts:
            self.starts.append(self.starts[-1] + c)

    @property
    def n(self) -> int:
        return self.starts[-1]

    def lower_bound(self, key: tuple) -> int:
        """First global index whose key is not below `key`: inside the last
        block whose first key is below it (one block read)."""
        j = -1
        for i, fk in enumerate(self.first_keys):  # index-block keys: host, tiny
            if fk < key:
                j = i
            else:
                break
        if j < 0:
            return 0
        return self.starts[j] + lower_bound(self.keys(j), self.counts[j], key)

    @classmethod
    def from_values(cls, limbs: list, n: int, block_values: int) -> "BlockedSide":
        """A side whose values are host arrays (tests and tools)."""
        starts = list(range(0, n, block_values))
        counts = [min(block_values, n - s) for s in starts]
        first = [_key(limbs, s) for s in starts]
        return cls(first, counts, lambda j: [l[starts[j]:starts[j] + counts[j]] for l in limbs])


def block_splitters(a: BlockedSide, b: BlockedSide, world: int) -> list:
    """P-1 splitter keys: data-block first keys of A ∪ B (index-block data
    only), the p-th being the first whose blocks before it hold at least
    p/world of the values. Identical on every rank."""
    blocks = sorted([(k, c) for k, c in zip(a.first_keys, a.counts)] + [(k, c) for k, c in zip(b.first_keys, b.counts)])
    total = a.n + b.n
    out, acc, i = [], 0, 0
    for p in range(1, world):
        goal = p * total // world
        while i < len(blocks) and acc + blocks[i][1] <= goal:
            acc += blocks[i][1]
            i += 1
        # the block that would cross the goal starts the next range (or the end: nothing left)
        out.append(blocks[i][0] if i < len(blocks) else None)
    return out


def block_cuts(a: BlockedSide, b: BlockedSide, splitters: list) -> list:
    """[(a_cut, b_cut)] * (world + 1) from the splitter keys: each cut is the
    splitter's lower bound in A and in B, so every value with that key (and
    every equal key) falls to the same rank. Cuts never move backwards."""
    cuts = [(0, 0)]
    for s in splitters:
        if s is None:
            cuts.append((a.n, b.n))
            continue
        pa, pb = cuts[-1]
        cuts.append((max(a.lower_bound(s), pa), max(b.lower_bound(s), pb)))
    cuts.append((a.n, b.n))
    return cuts


def rank_blocks(side: BlockedSide, lo: int, hi: int) -> list:
    """[(block, start, count)]: the parts of data blocks holding the side's
    global values [lo, hi) — all a rank stages of that side."""
    out = []
    for j, c in enumerate(side.counts):
        s = side.starts[j]
        x, y = max(lo, s), min(hi, s + c)
        if x < y:
            out.append((j, x - s, y - x))
    return out


def staged_bytes(cuts: list, rank: int, value_size: int) -> int:
    """Input bytes rank `rank` stages: its own range of A and B, nothing else."""
    (a0, b0), (a1, b1) = cuts[rank], cuts[rank + 1]
    return ((a1 - a0) + (b1 - b0)) * value_size


def range_segments(counts: list, lo: int, hi: int) -> list:
    """Pieces [(segment, start, count)] of the global index range [lo, hi) of a
    concatenation of segments with the given counts."""
    out, base = [], 0
    for s, n in enumerate(counts):
        a, b = max(lo, base), min(hi, base + n)
        if a < b:
            out.append((s, a - base, b - a))
        base += n
    return out


# ---------------------------------------------------------------------------
# Output ownership after the count exchange (pure arithmetic, same on every rank).

def data_block_slot(k: int, dbcm: int) -> int:
    """Acquire-order slot of data block k (tbc_internal.h data_block_slot)."""
    return k + k // dbcm


def index_block_slot(t: int, k_last: int) -> int:
    """Slot of the index block of table t whose last data block is k_last."""
    return k_last + t + 1


@dataclass
class SplitPlan:
    counts: list   # survivors of each rank's key range
    offsets: list  # global output position of each rank's first survivor
    total: int     # survivors of the whole job
    vcm: int
    dbcm: int

    @property
    def data_blocks(self) -> int:
        return -(-self.total // self.vcm)

    @property
    def table_count(self) -> int:
        return -(-self.data_blocks // self.dbcm)

    def blocks(self, p: int) -> tuple:
        """[k0, k1): the data blocks whose first value is rank p's (it finishes them)."""
        o, c = self.offsets[p], self.counts[p]
        k0, k1 = -(-o // self.vcm), -(-(o + c) // self.vcm)
        return (k0, max(k0, k1))

    def tables(self, p: int) -> tuple:
        """[t0, t1): the tables whose first data block is rank p's (it seals them)."""
        k0, k1 = self.blocks(p)
        return (-(-k0 // self.dbcm), -(-k1 // self.dbcm))

    def head(self, p: int) -> tuple:
        """(position, count): rank p's survivors inside a block an earlier rank owns."""
        o, c = self.offsets[p], self.counts[p]
        k0 = -(-o // self.vcm)
        return (o, min(k0 * self.vcm, o + c) - o)

    def block_owner(self, k: int) -> int:
        pos = k * self.vcm
        for p in range(len(self.counts)):
            if self.counts[p] and self.offsets[p] <= pos < self.offsets[p] + self.counts[p]:
                return p
        raise ValueError(f"block {k} is outside the job's output")

    def table_owner(self, t: int) -> int:
        return self.block_owner(t * self.dbcm)

    def entries(self, p: int) -> tuple:
        """(table, first slot, count): index entries of rank p's blocks that
        belong to a table an earlier rank owns (at most one table)."""
        k0, k1 = self.blocks(p)
        if k0 == k1 or k0 % self.dbcm == 0:
            return (k0 // self.dbcm, k0 % self.dbcm, 0)
        return (k0 // self.dbcm, k0 % self.dbcm, min(k1, (k0 // self.dbcm + 1) * self.dbcm) - k0)

    def k_last(self, t: int) -> int:
        return min((t + 1) * self.dbcm, self.data_blocks) - 1

    @property
    def head_max(self) -> int:
        return max((self.head(p)[1] for p in range(len(self.counts))), default=0)

    @property
    def entries_max(self) -> int:
        return max((self.entries(p)[2] for p in range(len(self.counts))), default=0)


def plan_split(counts: list, vcm: int, dbcm: int) -> SplitPlan:
    offsets, o = [], 0
    for c in counts:
        offsets.append(o)
        o += int(c)
    return SplitPlan([int(c) for c in counts], offsets, o, vcm, dbcm)


def entry_ranges(image: int, s0: int, e: int, dbcm: int, key_size: int) -> list:
    """[(address, bytes)]: index entries [s0, s0 + e) of an index block image
    (TableIndex layout, schema.zig:80-260): checksums (32 bytes each),
    keys_min, keys_max, addresses — four contiguous pieces."""
    ks = key_size
    cks, kmin = HEADER_SIZE, HEADER_SIZE + 32 * dbcm
    kmax, addr = kmin + ks * dbcm, kmin + 2 * ks * dbcm
    return [(image + cks + 32 * s0, 32 * e), (image + kmin + ks * s0, ks * e), (image + kmax + ks * s0, ks * e),
            (image + addr + 8 * s0, 8 * e)]


def entry_bytes(key_size: int) -> int:
    return 32 + 2 * key_size + 8


# ---------------------------------------------------------------------------
# The exchange (torch.distributed: RCCL over xGMI with "nccl", gloo on CPU).

class TorchExchange:
    """All-gathers of a split step over torch.distributed.

    On device (nccl: RCCL over xGMI, `device` a cuda device) every exchange is
    a collective enqueued on the ENGINE stream (torch.cuda.ExternalStream over
    tbc_engine_stream): the count merge writes its count into a device word,
    the counts are all-gathered behind it, and the one host wait of the step
    is reading the gathered counts (the host computes the plan from them).
    Heads and index entries are copied into exchange buffers, all-gathered
    and copied into place all in engine-stream order, with no host wait.
    Over gloo (host tensors; the CPU tests and a rehearsal with ranks sharing
    one GPU) each exchange goes through host memory."""

    def __init__(self, dist, device=None):
        self.dist, self.device = dist, device
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.on_device = device is not None and str(device).startswith("cuda")

    def _stream(self, engine):
        import torch
        return torch.cuda.ExternalStream(engine.stream_handle(), device=self.device)

    def _alloc(self, n: int, dtype):
        """A device tensor the engine stream writes: allocated (on torch's
        stream) and made ready before any engine-stream work touches it —
        the engine stream does not wait for torch's streams."""
        import torch
        t = torch.empty(n, dtype=dtype, device=self.device)
        torch.cuda.current_stream(self.device).synchronize()
        return t

    def count_buffer(self, engine, scratch: dict):
        """Where the count merge stores its count (device, u64)."""
        if self.on_device:
            import torch
            t = scratch.get("count_t")
            if t is None:
                t = scratch["count_t"] = self._alloc(2, torch.int64)
            return _Ptr(t.data_ptr())
        buf = scratch.get("count_buf")
        if buf is None:
            buf = scratch["count_buf"] = engine.alloc(256)
        return buf

    def gather_counts(self, engine, count_batch, count_buf, scratch: dict) -> list:
        import torch
        if self.on_device:
            out = scratch.get("counts_t")
            if out is None:
                out = scratch["counts_t"] = self._alloc(self.world, torch.int64)
            with torch.cuda.stream(self._stream(engine)):
                self.dist.all_gather_into_tensor(out, scratch["count_t"][:1])
                return [int(x) for x in out.cpu()]  # the step's one host wait
        count_batch.wait()
        t = torch.tensor([int(count_batch.result(0)[0].value_count)], dtype=torch.int64)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def all_gather_bytes(self, engine, segments: list, nbytes: int, key: str, scratch: dict):
        """All-gather each rank's bytes (`segments`, device, <= nbytes) into
        per-rank device buffers. Returns (keep-alive objects, [ptr per rank])."""
        import torch
        if nbytes == 0:
            return [], [0] * self.world
        if self.on_device:
            mine, out = scratch.get(key + "_mine"), scratch.get(key + "_out")
            if mine is None or mine.numel() < nbytes:
                mine = scratch[key + "_mine"] = self._alloc(nbytes, torch.uint8)
                out = scratch[key + "_out"] = self._alloc(self.world * nbytes, torch.uint8)
            copies, off = [], 0
            for ptr, n in segments:
                copies.append((mine.data_ptr() + off, ptr, n))
                off += n
            if copies:
                engine.copy_device_batch(copies)  # engine stream, after the bodies
            with torch.cuda.stream(self._stream(engine)):
                self.dist.all_gather_into_tensor(out[:self.world * nbytes], mine[:nbytes])
            return [mine, out], [out.data_ptr() + q * nbytes for q in range(self.world)]
        host = np.zeros(nbytes, dtype=np.uint8)
        staging = engine.alloc(nbytes)
        off = 0
        for ptr, n in segments:
            engine.copy_device_async(staging.ptr + off, ptr, n)
            off += n
        # The download waits for the engine stream (the copies above, after
        # the bodies) and the last seal (the entries it wrote), not for other
        # batches' tails.
        host[:] = staging.download(nbytes)
        mine = torch.from_numpy(host)
        out = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(out, mine)
        bufs = [engine.upload(x.numpy()) for x in out]
        return bufs, [b.ptr for b in bufs]


class SingleRank:
    """The exchange of a world of one (no communication)."""
    rank, world = 0, 1

    def count_buffer(self, engine, scratch: dict):
        buf = scratch.get("count_buf")
        if buf is None:
            buf = scratch["count_buf"] = engine.alloc(256)
        return buf

    def gather_counts(self, engine, count_batch, count_buf, scratch: dict) -> list:
        count_batch.wait()
        return [int(count_batch.result(0)[0].value_count)]

    def all_gather_bytes(self, engine, segments: list, nbytes: int, key: str, scratch: dict):
        assert nbytes == 0
        return [], [0]


@dataclass
class _Ptr:
    ptr: int


# ---------------------------------------------------------------------------
# One rank's part of a split job on its GPU.

@dataclass
class SplitResult:
    blocks: tuple          # (k0, k1): the job's data blocks this rank finished
    tables: tuple          # (t0, t1): the job's tables this rank sealed
    plan: SplitPlan
    exchanged: dict        # bytes this rank sent per exchange: counts, heads, entries
    arena: object          # DeviceBuffer: this rank's slots [base_slot, base_slot + arena.nbytes / block_size)
    base_slot: int
    block_size: int
    pending: list          # enqueued batches (count merge, bodies, seals), waited for by finish()
    table_batch: object = None
    keep: list = None      # exchange buffers the enqueued copies read
    result: object = None  # tbc_compaction_result of the sealing of the tables (finish; None if none)
    table_infos: np.ndarray = None

    def slot_ptr(self, slot: int) -> int:
        """Device address of the job's output slot `slot` (one this rank holds)."""
        assert self.base_slot <= slot < self.base_slot + self.arena.nbytes // self.block_size, slot
        return self.arena.ptr + (slot - self.base_slot) * self.block_size

    def finish(self) -> "SplitResult":
        """Wait for the step's enqueued work; the sealed tables' result and
        TableInfos."""
        for b in self.pending:
            b.wait()
        self.table_infos = np.zeros((0, 128), dtype=np.uint8)
        if self.table_batch is not None:
            self.result, self.table_infos = self.table_batch.result(0)
            if self.result.status != 0:
                raise RuntimeError(f"split seal: status {self.result.status}")
        for b in self.pending:
            b.release()
        self.pending, self.keep = [], None
        return self


def slot_range(plan: SplitPlan, p: int) -> tuple:
    """[lo, hi): the output slots rank p writes — the data blocks its
    survivors fall in (the head block an earlier rank owns included) and the
    index blocks of the tables its blocks belong to (which may lie past its
    blocks, inside the next rank's range)."""
    o, c = plan.offsets[p], plan.counts[p]
    if c == 0:
        return (0, 1)
    vcm, dbcm = plan.vcm, plan.dbcm
    lo = data_block_slot(o // vcm, dbcm)
    hi = data_block_slot((o + c - 1) // vcm, dbcm)
    k0, k1 = plan.blocks(p)
    if k1 > k0:
        for t in range(k0 // dbcm, (k1 - 1) // dbcm + 1):
            hi = max(hi, index_block_slot(t, plan.k_last(t)))
    return (lo, hi + 1)


def compact_split(engine, job, cuts: list, exchange, rank: int, staged: bool = False, scratch: dict | None = None,
                  before_phase2=None) -> SplitResult:
    """Enqueue rank `rank`'s share of `job` split at `cuts` (block_cuts or
    split_points); call `.finish()` on the result to wait for it. With
    staged=True the job's segments hold only this rank's range
    [cuts[rank], cuts[rank+1]) of A and of B (what rank_blocks named, staged
    on this GPU); otherwise the whole job's inputs, sliced here. `scratch` (a
    dict kept by a caller that repeats the split) keeps the output slots and
    exchange buffers between steps; `before_phase2` runs once the bodies,
    the partial blocks and the data-block seal are enqueued (a caller enqueues
    its other work there: the seal's chains run on a tail stream beside it).

    Host waits: one, reading the gathered counts (the plan — every offset,
    block and table range — is host arithmetic on them), when the exchange
    is on the device; everything after that is enqueued on the engine stream
    (bodies, heads, seals, entries, seals). An exchange through host memory
    (gloo) also waits before each of its two byte all-gathers.

    The rank holds only its own output slots (`slot_range`): the job's
    output_blocks base handed to the engine is that allocation minus the
    slots before it, and the engine touches no slot outside the range."""
    from .abi import COMPACTION_COUNT_ONLY
    from .engine import Job
    tree, bs = job.tree, engine.block_size
    lay = engine.layout(tree)
    vcm, dbcm, vs, ks = lay.block_value_count_max, lay.data_block_count_max, tree.value_size, tree.key_size
    addrs = np.asarray(job.addresses, dtype=np.uint64)
    scratch = {} if scratch is None else scratch

    def sub(segs, lo, hi):
        return [(segs[s][0] + st * vs, n) for s, st, n in range_segments([n for _, n in segs], lo, hi)]

    (a_lo, b_lo), (a_hi, b_hi) = cuts[rank], cuts[rank + 1]
    if staged:
        seg_a, seg_b = list(job.segments_a), list(job.segments_b)
        assert sum(n for _, n in seg_a) == a_hi - a_lo and sum(n for _, n in seg_b) == b_hi - b_lo, \
            "staged segments are not this rank's range"
    else:
        seg_a, seg_b = sub(job.segments_a, a_lo, a_hi), sub(job.segments_b, b_lo, b_hi)

    def job_of(flags, output, offset=0, addresses=addrs):
        return Job(tree, seg_a, seg_b, job.a_immutable, job.drop_tombstones, job.level_b, job.cluster,
                   job.snapshot_min, addresses, output, flags=flags, output_offset=offset)

    # Counts (the merge alone, its count into a device word), then every
    # rank's global output offset.
    count_buf = exchange.count_buffer(engine, scratch)
    b0 = engine.submit([job_of(COMPACTION_COUNT_ONLY, count_buf, addresses=addrs[:0])])
    pending = [b0]
    plan = plan_split(exchange.gather_counts(engine, b0, count_buf, scratch), vcm, dbcm)
    sent = {"counts": 8, "heads": 0, "entries": 0}
    lo, hi = slot_range(plan, rank)
    arena = scratch.get("arena")
    if arena is None or arena.nbytes < (hi - lo) * bs:
        arena = scratch["arena"] = engine.alloc((hi - lo) * bs)
    out = _Ptr(arena.ptr - lo * bs)  # slot 0 of the job's layout

    # Bodies at their global positions in the job's own block layout.
    if plan.counts[rank]:
        pending.append(engine.submit([job_of(VALUES_ONLY, out, plan.offsets[rank])]))

    def position_ptr(pos: int) -> int:
        k = pos // vcm
        return out.ptr + data_block_slot(k, dbcm) * bs + HEADER_SIZE + (pos - k * vcm) * vs

    # The partial block's values to its owner.
    pos, h = plan.head(rank)
    sent["heads"] = h * vs
    keep1, ptrs = exchange.all_gather_bytes(engine, [(position_ptr(pos), h * vs)] if h else [],
                                            plan.head_max * vs, "heads", scratch)
    copies = []
    for q in range(len(plan.counts)):
        qpos, qh = plan.head(q)
        if q != rank and qh and plan.block_owner(qpos // vcm) == rank:
            copies.append((position_ptr(qpos), ptrs[q], qh * vs))
    if copies:
        engine.copy_device_batch(copies)
    k0, k1 = plan.blocks(rank)
    t0, t1 = plan.tables(rank)

    def seal(blocks, tables):
        return engine.seal_submit(tree, job.cluster, job.snapshot_min, job.level_b, addrs, out, plan.total, blocks,
                                  tables)

    if k1 > k0:
        pending.append(seal((k0, k1), (t0, t0)))
    # The caller's other work (the rank's whole jobs) goes on the engine
    # stream here: the data-block seal's chains run on a tail beside it, and
    # an exchange through host memory waits for it only at the entries.
    if before_phase2 is not None:
        before_phase2()
    # The index entries of a table an earlier rank owns, to that owner.
    t, s0, e = plan.entries(rank)
    sent["entries"] = e * entry_bytes(ks)
    mine = []
    if e:
        mine = entry_ranges(out.ptr + index_block_slot(t, plan.k_last(t)) * bs, s0, e, dbcm, ks)
    keep2, ptrs = exchange.all_gather_bytes(engine, mine, plan.entries_max * entry_bytes(ks), "entries", scratch)
    copies = []
    for q in range(len(plan.counts)):
        qt, qs0, qe = plan.entries(q)
        if q != rank and qe and plan.table_owner(qt) == rank:
            image = out.ptr + index_block_slot(qt, plan.k_last(qt)) * bs
            off = 0
            for dst, n in entry_ranges(image, qs0, qe, dbcm, ks):
                copies.append((dst, ptrs[q] + off, n))
                off += n
    if copies:
        engine.copy_device_batch(copies)
    table_batch = None
    if t1 > t0:
        table_batch = seal((k0, k0), (t0, t1))
        pending.append(table_batch)
    return SplitResult((k0, k1), (t0, t1), plan, sent, arena, lo, bs, pending, table_batch, [keep1, keep2])
