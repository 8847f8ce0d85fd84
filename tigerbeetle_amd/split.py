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
2. Phase 1: each rank compacts its key range values-only (bodies in scratch
   data-block slots, no headers or checksums) and takes its survivor count c_p.
3. Exchange (the only collective): all-gather of the counts c_p, then of each
   rank's head survivors — the ones the previous table owner still needs to
   complete a table that starts before this rank's range (≤ one table).
4. Phase 2: rank p owns the output tables whose first survivor is its own and
   re-blocks them: a compaction whose disk A is exactly those survivors (own
   tail + received heads) and whose B is empty writes every value unchanged
   (copy(.a), compaction.zig:786-804), with the job's addresses for those
   tables. The blocks, index blocks, checksums and TableInfos are therefore
   byte-identical to the unsplit job's (tested against the oracle).

Phase 1 runs with TBC_COMPACTION_VALUES_ONLY (merge + body assembly, no AEGIS
chains or index blocks), so the split costs one extra HBM pass over the
survivors, not a second set of checksums. Splitting one job pays off only when
a job is larger than a GPU's share of the half-bar, which no BASELINE config
needs.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .abi import COMPACTION_VALUES_ONLY

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
# Output ownership after the count exchange.

@dataclass
class TablePlan:
    offsets: list          # global index of each rank's first survivor
    total: int             # survivors of the whole job
    table_values: int      # values per full table (vcm · dbcm)
    tables: list           # [(t0, t1)] tables owned by each rank
    need: list             # head survivors each rank must send (to earlier owners)

    @property
    def head_max(self) -> int:
        return max(self.need) if self.need else 0

    def stream(self, rank: int) -> list:
        """Rank `rank`'s phase-2 input as [(source rank, local start, count)]:
        its own survivors from its first owned table on, then heads of the
        following ranks up to the end of its last owned table."""
        t0, t1 = self.tables[rank]
        if t0 == t1:
            return []
        T = self.table_values
        start, end = t0 * T, min(t1 * T, self.total)
        out = []
        for q in range(rank, len(self.offsets)):
            o = self.offsets[q]
            c = (self.offsets[q + 1] if q + 1 < len(self.offsets) else self.total) - o
            a, b = max(start, o), min(end, o + c)
            if a < b:
                assert q == rank or (a == o and b - a <= self.need[q]), "stream exceeds the exchanged head"
                out.append((q, a - o, b - a))
            if o + c >= end:
                break
        return out


def plan_tables(counts: list, vcm: int, dbcm: int) -> TablePlan:
    T = vcm * dbcm
    offsets, o = [], 0
    for c in counts:
        offsets.append(o)
        o += int(c)
    total = o
    tables, need = [], []
    for o_p, c in zip(offsets, counts):
        tables.append((-(-o_p // T), -(-(o_p + c) // T)))
        need.append(min(int(c), T - o_p % T) if c and o_p % T else 0)
    return TablePlan(offsets, total, T, tables, need)


def table_address_range(t0: int, t1: int, total: int, vcm: int, dbcm: int) -> tuple:
    """Indices [lo, hi) of tables t0..t1-1 in the job's acquire-order address
    list: each full table is dbcm data blocks then its index block."""
    T = vcm * dbcm
    lo = t0 * (dbcm + 1)
    if t0 == t1:
        return lo, lo
    n = min(t1 * T, total) - t0 * T
    db = -(-n // vcm)
    return lo, lo + db + (t1 - t0)


def survivor_segments(out_ptr: int, count: int, vcm: int, dbcm: int, value_size: int, block_size: int) -> list:
    """Device segments [(ptr, count)] of a compaction's survivors inside its
    output arena (data block k in slot k + k // dbcm, values at +256)."""
    segs = []
    for k in range(-(-count // vcm)):
        slot = k + k // dbcm
        segs.append((out_ptr + slot * block_size + HEADER_SIZE, min(vcm, count - k * vcm)))
    return segs


# ---------------------------------------------------------------------------
# The exchange (torch.distributed: RCCL over xGMI with "nccl", gloo on CPU).

class TorchExchange:
    def __init__(self, dist, device=None):
        self.dist, self.device = dist, device
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def all_gather_counts(self, count: int) -> list:
        import torch
        t = torch.tensor([count], dtype=torch.int64, device=self.device)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def all_gather_heads(self, engine, segments: list, nbytes: int):
        """All-gather each rank's head (`segments`, device, ≤ nbytes) into
        per-rank device buffers. Returns (keep-alive objects, [ptr per rank])."""
        import torch
        if nbytes == 0:
            return [], [0] * self.world
        on_device = self.device is not None and str(self.device).startswith("cuda")
        if on_device:
            mine = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
            torch.cuda.synchronize(self.device)
            off = 0
            for ptr, n in segments:
                engine.copy_device_async(mine.data_ptr() + off, ptr, n)
                off += n
            engine.synchronize()
            out = [torch.empty_like(mine) for _ in range(self.world)]
            self.dist.all_gather(out, mine)
            torch.cuda.synchronize(self.device)
            return out, [x.data_ptr() for x in out]
        host = np.zeros(nbytes, dtype=np.uint8)
        staging = engine.alloc(nbytes)
        off = 0
        for ptr, n in segments:
            engine.copy_device_async(staging.ptr + off, ptr, n)
            off += n
        engine.synchronize()
        host[:] = staging.download(nbytes)
        mine = torch.from_numpy(host)
        out = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(out, mine)
        bufs = [engine.upload(x.numpy()) for x in out]
        return bufs, [b.ptr for b in bufs]


class SingleRank:
    """The exchange of a world of one (no communication)."""
    rank, world = 0, 1

    def all_gather_counts(self, count: int) -> list:
        return [count]

    def all_gather_heads(self, engine, segments: list, nbytes: int):
        assert nbytes == 0
        return [], [0]


# ---------------------------------------------------------------------------
# One rank's part of a split job on its GPU.

@dataclass
class SplitResult:
    tables: tuple          # (t0, t1): the job's output tables this rank wrote
    result: object         # tbc_compaction_result of phase 2 (None if no tables)
    table_infos: np.ndarray
    blocks: object         # DeviceBuffer of the phase-2 output arena (None if no tables)
    plan: TablePlan


def compact_split(engine, job, cuts: list, exchange, rank: int, staged: bool = False, scratch: dict | None = None,
                  before_phase2=None) -> SplitResult:
    """Run rank `rank`'s share of `job` split at `cuts` (block_cuts or
    split_points). With staged=True the job's segments hold only this rank's
    range [cuts[rank], cuts[rank+1]) of A and of B (what rank_blocks named,
    staged on this GPU); otherwise the whole job's inputs, sliced here.
    `scratch` (a dict kept by a caller that repeats the split) keeps the two
    output arenas between calls; `before_phase2` runs after the exchange, just
    before phase 2 is submitted (a caller enqueues its other work there)."""
    from .engine import Job
    tree, bs = job.tree, engine.block_size

    def arena(name: str, nbytes: int):
        if scratch is None:
            return engine.alloc(nbytes)
        buf = scratch.get(name)
        if buf is None or buf.nbytes < nbytes:
            buf = scratch[name] = engine.alloc(nbytes)
        return buf
    lay = engine.layout(tree)
    vcm, dbcm, vs = lay.block_value_count_max, lay.data_block_count_max, tree.value_size

    def sub(segs, lo, hi):
        return [(segs[s][0] + st * vs, n) for s, st, n in range_segments([n for _, n in segs], lo, hi)]

    (a_lo, b_lo), (a_hi, b_hi) = cuts[rank], cuts[rank + 1]
    if staged:
        seg_a, seg_b = list(job.segments_a), list(job.segments_b)
        assert sum(n for _, n in seg_a) == a_hi - a_lo and sum(n for _, n in seg_b) == b_hi - b_lo, \
            "staged segments are not this rank's range"
    else:
        seg_a, seg_b = sub(job.segments_a, a_lo, a_hi), sub(job.segments_b, b_lo, b_hi)
    n = (a_hi - a_lo) + (b_hi - b_lo)
    db = -(-n // vcm)
    nblocks = db + -(-db // dbcm)
    out1 = arena("phase1", max(1, nblocks) * bs)
    p1 = Job(tree, seg_a, seg_b, job.a_immutable, job.drop_tombstones, job.level_b, job.cluster,
             job.snapshot_min, np.arange(1, nblocks + 1, dtype=np.uint64), out1, flags=COMPACTION_VALUES_ONLY)
    b1 = engine.submit([p1])
    b1.wait()
    r1, _ = b1.result(0)
    b1.release()
    if r1.status != 0:
        raise RuntimeError(f"split phase 1 failed on rank {rank}: status {r1.status}")
    mine = survivor_segments(out1.ptr, r1.value_count, vcm, dbcm, vs, bs)

    plan = plan_tables(exchange.all_gather_counts(int(r1.value_count)), vcm, dbcm)
    head = [(p, c * vs) for p, c in sub(mine, 0, plan.need[rank])]
    keep, head_ptrs = exchange.all_gather_heads(engine, head, plan.head_max * vs)

    if before_phase2 is not None:
        before_phase2()
    t0, t1 = plan.tables[rank]
    if t0 == t1:
        return SplitResult((t0, t1), None, np.zeros((0, 128), dtype=np.uint8), None, plan)
    seg2 = []
    for q, st, cnt in plan.stream(rank):
        if q == rank:
            seg2 += sub(mine, st, st + cnt)
        else:  # received head, in segments of at most one block's values
            seg2 += [(head_ptrs[q] + (st + k) * vs, min(vcm, cnt - k)) for k in range(0, cnt, vcm)]
    lo, hi = table_address_range(t0, t1, plan.total, vcm, dbcm)
    addrs = np.asarray(job.addresses, dtype=np.uint64)[lo:hi]
    if len(addrs) != hi - lo:
        raise ValueError("address list shorter than the job's output")
    out2 = arena("phase2", (hi - lo) * bs)
    p2 = Job(tree, seg2, [], False, False, job.level_b, job.cluster, job.snapshot_min, addrs, out2)
    b2 = engine.submit([p2])
    b2.wait()
    r2, infos = b2.result(0)
    b2.release()
    del keep
    if r2.status != 0 or r2.table_count != t1 - t0:
        raise RuntimeError(f"split phase 2 failed on rank {rank}: status {r2.status}")
    if scratch is None:
        out1.free()
    return SplitResult((t0, t1), r2, infos, out2, plan)
