"""Key-range split of one compaction across ranks (tigerbeetle_amd/split.py,
SURVEY.md §8e.2) on CPU: the splitters, the count exchange, table ownership
and the head exchange, with the oracle standing in for each rank's GPU
compaction. The re-blocked tables must equal the unsplit job's output byte for
byte (blocks, index blocks, checksums, TableInfos)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import data_values_from_blocks, disk_image, oracle_tree
from tigerbeetle_amd import split, trees, workloads

BS = 4096
CLUSTER, SNAPSHOT_MIN, LEVEL_B = 0xC1, 48, 2


def small_tree(name, tables=3):
    base = trees.BY_NAME[name]
    return trees.with_table_size(base, tables * (BS - 256) // base.value_size + 5)


CASES = [
    ("transfers.id", dict(n_a=700, b_table_sizes=[400, 380, 390], a_immutable=True, dup_frac=0.1, overlap=0.3)),
    ("transfers.id", dict(n_a=900, b_table_sizes=[500, 450], a_immutable=False, tomb_frac=0.05,
                          drop_tombstones=True)),
    ("accounts.timestamp", dict(n_a=150, b_table_sizes=[90, 80], a_immutable=True, dup_frac=0.3, tomb_frac=0.1,
                                drop_tombstones=True, overlap=0.5)),
    ("transfers.debit_account_id", dict(n_a=1500, b_table_sizes=[700, 600], a_immutable=True, dup_frac=0.2,
                                        overlap=0.2)),
    ("accounts.ledger", dict(n_a=2000, b_table_sizes=[900], a_immutable=False, overlap=0.4)),
]


def _inputs(i):
    name, kw = CASES[i]
    spec = small_tree(name)
    rng = np.random.default_rng(0x5EED + i)
    ji = workloads.make_job_inputs(spec, rng, **kw)
    n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n, BS) + 2, rng, 1000, 0.1)
    return spec, ji, addrs


def _b_all(ji):
    vs = ji.tree.value_size
    return np.concatenate(ji.b_tables) if ji.b_tables else np.zeros((0, vs), np.uint8)


def _compact(oracle, spec, a, a_immutable, b, drop, addrs):
    t = oracle_tree(oracle, spec, BS)
    vcm = t.block_value_count_max
    a_segs = ([a] if len(a) else []) if a_immutable else workloads.split_blocks(a, vcm)
    r = oracle.compact(t, a_segs, workloads.split_blocks(b, vcm), a_immutable=a_immutable, drop_tombstones=drop,
                       level_b=LEVEL_B, cluster=CLUSTER, snapshot_min=SNAPSHOT_MIN, addresses=addrs)
    assert r.status == 0
    return r


def _rank_phase1(oracle, spec, ji, cuts, rank):
    (a_lo, b_lo), (a_hi, b_hi) = cuts[rank], cuts[rank + 1]
    a, b = ji.a_values[a_lo:a_hi], _b_all(ji)[b_lo:b_hi]
    n = len(a) + len(b)
    scratch = np.arange(1, workloads.worst_case_blocks(spec, max(n, 1), BS) + 1, dtype=np.uint64)
    r = _compact(oracle, spec, a, ji.a_immutable, b, ji.drop_tombstones, scratch)
    return data_values_from_blocks(r.blocks[: len(r.blocks)], spec.value_size)


def _rank_phase2(oracle, spec, plan, rank, survivors_of, addrs):
    """Re-block rank's owned tables from its survivors and the exchanged heads."""
    lay = spec.layout(BS)
    t0, t1 = plan.tables[rank]
    if t0 == t1:
        return [], np.zeros((0, 128), np.uint8)
    stream = np.concatenate([survivors_of(q)[st:st + c] for q, st, c in plan.stream(rank)])
    lo, hi = split.table_address_range(t0, t1, plan.total, lay["block_value_count_max"],
                                       lay["data_block_count_max"])
    r = _compact(oracle, spec, stream, False, stream[:0], False, addrs[lo:hi])
    assert len(r.table_infos) == t1 - t0
    return [disk_image(b) for b in r.blocks], r.table_infos


def _cuts(spec, ji, world):
    b = _b_all(ji)
    la, lb = workloads.keys_of(ji.a_values, spec), workloads.keys_of(b, spec)
    return split.split_points(la, len(ji.a_values), lb, len(b), world)


def _sides(spec, ji, reads=None):
    """A and B as data blocks (first keys from the 'index blocks'); `reads`
    collects every (side, block) whose keys are read."""
    vcm = spec.layout(BS)["block_value_count_max"]
    out = []
    for name, vals in (("a", ji.a_values), ("b", _b_all(ji))):
        side = split.BlockedSide.from_values(workloads.keys_of(vals, spec), len(vals), vcm)
        if reads is not None:
            inner = side.keys
            side.keys = (lambda nm, f: (lambda j: (reads.append((nm, j)), f(j))[1]))(name, inner)
        out.append(side)
    return out


def _block_cuts(spec, ji, world, reads=None):
    a, b = _sides(spec, ji, reads)
    return split.block_cuts(a, b, split.block_splitters(a, b, world))


@pytest.mark.parametrize("case", range(len(CASES)))
def test_split_points_never_split_a_key(case):
    spec, ji, _ = _inputs(case)
    b = _b_all(ji)
    na, nb = len(ji.a_values), len(b)
    ka = [tuple(k) for k in np.stack(workloads.keys_of(ji.a_values, spec), 1)[:, ::-1].tolist()]
    kb = [tuple(k) for k in np.stack(workloads.keys_of(b, spec), 1)[:, ::-1].tolist()]
    for world in (1, 2, 3, 4, 8):
        cuts = _cuts(spec, ji, world)
        assert cuts[0] == (0, 0) and cuts[-1] == (na, nb)
        for p in range(1, world):
            (a, bc) = cuts[p]
            assert cuts[p - 1][0] <= a and cuts[p - 1][1] <= bc
            left = ([ka[a - 1]] if a else []) + ([kb[bc - 1]] if bc else [])
            right = ([ka[a]] if a < na else []) + ([kb[bc]] if bc < nb else [])
            if left and right:
                assert max(left) < min(right), "a key straddles two ranks"
        sizes = [cuts[p + 1][0] - cuts[p][0] + cuts[p + 1][1] - cuts[p][1] for p in range(world)]
        assert sum(sizes) == na + nb
        if world > 1 and not ji.a_immutable:  # unique keys: balanced to within a key run
            assert max(sizes) - min(sizes) <= 2 + (na + nb) // world // 4


def test_plan_tables_edges():
    vcm, dbcm = 10, 3
    T = vcm * dbcm
    plan = split.plan_tables([0, 45, 0, 5, 31, 0], vcm, dbcm)
    assert plan.total == 81 and plan.offsets == [0, 0, 45, 45, 50, 81]
    assert plan.tables == [(0, 0), (0, 2), (2, 2), (2, 2), (2, 3), (3, 3)]
    assert plan.need == [0, 0, 0, 5, 10, 0]
    assert plan.stream(1) == [(1, 0, 45), (3, 0, 5), (4, 0, 10)]
    assert plan.stream(4) == [(4, 10, 21)]
    assert all(plan.stream(r) == [] for r in (0, 2, 3, 5))
    assert split.table_address_range(0, 2, 81, vcm, dbcm) == (0, 8)
    assert split.table_address_range(2, 3, 81, vcm, dbcm) == (8, 12)
    assert split.table_address_range(2, 3, 2 * T + 1, vcm, dbcm) == (8, 10)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_block_cuts_read_only_boundary_blocks(case, world):
    """Per-rank staging: the cuts come from the data blocks' first keys plus
    at most one block of A and one of B per splitter; no key straddles a
    cut; every rank stages about its share (its range, whole-block slack)."""
    spec, ji, _ = _inputs(case)
    reads = []
    cuts = _block_cuts(spec, ji, world, reads)
    assert len(reads) <= 2 * (world - 1)
    b = _b_all(ji)
    ka = [tuple(int(l[i]) for l in reversed(workloads.keys_of(ji.a_values, spec))) for i in range(len(ji.a_values))]
    kb = [tuple(int(l[i]) for l in reversed(workloads.keys_of(b, spec))) for i in range(len(b))]
    for (a0, b0), (a1, b1) in zip(cuts, cuts[1:]):
        assert a0 <= a1 and b0 <= b1
    for p in range(1, world):
        a_cut, b_cut = cuts[p]
        left = ka[:a_cut] + kb[:b_cut]
        right = ka[a_cut:] + kb[b_cut:]
        if left and right:
            assert max(left) < min(right)
    n, vs = len(ji.a_values) + len(b), spec.value_size
    vcm = spec.layout(BS)["block_value_count_max"]
    assert sum(split.staged_bytes(cuts, p, vs) for p in range(world)) == n * vs
    for p in range(world):
        assert split.staged_bytes(cuts, p, vs) <= (n // world + 2 * vcm * (world > 1) + 2 * vcm) * vs


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("method", ["merge_path", "blocks"])
def test_split_job_equals_unsplit_job(oracle_lib, case, world, method):
    spec, ji, addrs = _inputs(case)
    whole = _compact(oracle_lib, spec, ji.a_values, ji.a_immutable, _b_all(ji), ji.drop_tombstones, addrs)
    cuts = _cuts(spec, ji, world) if method == "merge_path" else _block_cuts(spec, ji, world)
    surv = [_rank_phase1(oracle_lib, spec, ji, cuts, p) for p in range(world)]
    lay = spec.layout(BS)
    plan = split.plan_tables([len(s) for s in surv], lay["block_value_count_max"], lay["data_block_count_max"])
    assert plan.total == whole.value_count
    images, infos = [], []
    for p in range(world):
        im, inf = _rank_phase2(oracle_lib, spec, plan, p, lambda q: surv[q], addrs)
        images += im
        infos.append(inf)
    expect = [disk_image(b) for b in whole.blocks]
    assert len(images) == len(expect)
    for g, w in zip(images, expect):
        assert np.array_equal(g, w)
    assert np.array_equal(np.concatenate(infos), whole.table_infos)


# --- the same flow with the exchange over gloo, world_size 2 and 3 -----------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    spec, ji, addrs = _inputs(case)
    reads = []
    cuts = _block_cuts(spec, ji, world, reads)      # identical on every rank, no communication
    assert len(reads) <= 2 * (world - 1)            # index keys + boundary blocks only
    mine = _rank_phase1(oracle, spec, ji, cuts, rank)  # stages only [cuts[rank], cuts[rank+1])
    ex = split.TorchExchange(dist)
    lay = spec.layout(BS)
    plan = split.plan_tables(ex.all_gather_counts(len(mine)), lay["block_value_count_max"],
                             lay["data_block_count_max"])
    vs = spec.value_size
    head = np.zeros((max(1, plan.head_max), vs), np.uint8)
    head[: plan.need[rank]] = mine[: plan.need[rank]]
    heads = [torch.empty(head.size, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(heads, torch.from_numpy(head.reshape(-1)))
    heads = [h.numpy().reshape(-1, vs) for h in heads]
    images, infos = _rank_phase2(oracle, spec, plan, rank, lambda r: mine if r == rank else heads[r], addrs)
    q.put((rank, [bytes(x) for x in images], infos.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, 0), (3, 3)])
def test_split_exchange_over_gloo(oracle_lib, world, case):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec, ji, addrs = _inputs(case)
    whole = _compact(oracle_lib, spec, ji.a_values, ji.a_immutable, _b_all(ji), ji.drop_tombstones, addrs)
    images = [im for _, ims, _ in out for im in ims]
    assert images == [bytes(disk_image(b)) for b in whole.blocks]
    assert b"".join(inf for _, _, inf in out) == whole.table_infos.tobytes()


# --- TorchExchange.all_gather_heads (host-staged gloo path) on CPU -----------

class _FakeBuffer:
    def __init__(self, mem, ptr, n):
        self.mem, self.ptr, self.nbytes = mem, ptr, n

    def download(self, n):
        return np.frombuffer(bytes(self.mem.read(self.ptr, n)), np.uint8)

    def free(self):
        pass


class _FakeMemory:
    """Flat byte-addressed stand-in for device memory (no GPU on this host)."""

    def __init__(self):
        self.heap = bytearray(1 << 20)
        self.top = 4096

    def alloc(self, n):
        p = self.top
        self.top += (n + 15) // 16 * 16
        return p

    def read(self, p, n):
        return self.heap[p:p + n]

    def write(self, p, b):
        self.heap[p:p + len(b)] = b


class _FakeEngine:
    def __init__(self):
        self.mem = _FakeMemory()

    def alloc(self, n):
        return _FakeBuffer(self.mem, self.mem.alloc(n), n)

    def upload(self, a):
        b = self.alloc(a.nbytes)
        self.mem.write(b.ptr, a.tobytes())
        return b

    def copy_device_async(self, dst, src, n):
        self.mem.write(dst, bytes(self.mem.read(src, n)))

    def synchronize(self):
        pass


def _heads_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _FakeEngine()
    vals = np.arange(100, dtype=np.uint64).reshape(-1, 2).view(np.uint8) + rank  # 50 values of 16 B
    buf = eng.upload(vals)
    need = [0, 7, 3][rank]
    segs = [(buf.ptr, 16 * min(need, 4)), (buf.ptr + 64, 16 * max(0, need - 4))]  # head in two pieces
    ex = split.TorchExchange(dist)
    _, ptrs = ex.all_gather_heads(eng, [s for s in segs if s[1]], 7 * 16)
    got = [bytes(eng.mem.read(p, 7 * 16)) for p in ptrs]
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_heads_host_path_over_gloo():
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_heads_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        for q_ in range(world):
            need = [0, 7, 3][q_]
            vals = (np.arange(100, dtype=np.uint64).reshape(-1, 2).view(np.uint8) + q_).tobytes()
            assert out[r][q_][:16 * need] == vals[:16 * need]
            assert out[r][q_][16 * need:] == bytes(16 * (7 - need))
