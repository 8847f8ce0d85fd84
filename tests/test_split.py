"""Key-range split of one compaction across ranks (tigerbeetle_amd/split.py,
SURVEY.md §8e.2) on CPU: the splitters, then split.compact_split itself —
count exchange, bodies in place at global positions, the partial block's
values to its owner, data blocks finished in place, index entries to the
table's owner, index blocks sealed — run against an oracle-backed stand-in
for each rank's engine (the oracle merges each rank's key range; data and
index blocks are finished by a Python restatement of data_block_finish /
index_block_finish checked by the comparison itself). The union of the
ranks' data blocks, index blocks and TableInfos must equal the unsplit job's
output byte for byte, and each exchange must stay within one block's values
and one table's index entries per rank."""
import os
import socket
import threading
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import data_values_from_blocks, disk_image, oracle_tree
from oracle import oracle as _oracle
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



def test_plan_split_edges():
    vcm, dbcm = 10, 3
    plan = split.plan_split([0, 45, 0, 5, 31, 0], vcm, dbcm)
    assert plan.total == 81 and plan.offsets == [0, 0, 45, 45, 50, 81]
    assert plan.data_blocks == 9 and plan.table_count == 3
    assert [plan.blocks(p) for p in range(6)] == [(0, 0), (0, 5), (5, 5), (5, 5), (5, 9), (9, 9)]
    assert [plan.tables(p) for p in range(6)] == [(0, 0), (0, 2), (2, 2), (2, 2), (2, 3), (3, 3)]
    # rank 1's last block (40..49) takes 5 values from rank 3 and 0 from rank 4 (it starts block 5)
    assert [plan.head(p) for p in range(6)] == [(0, 0), (0, 0), (45, 0), (45, 5), (50, 0), (81, 0)]
    assert plan.block_owner(4) == 1 and plan.block_owner(5) == 4 and plan.table_owner(1) == 1
    # rank 4 finishes blocks 5..8: block 5 belongs to table 1 (rank 1's)
    assert plan.entries(4) == (1, 2, 1) and plan.entries(1) == (0, 0, 0)
    assert plan.k_last(2) == 8 and plan.head_max == 5 and plan.entries_max == 1
    solo = split.plan_split([7], 10, 3)
    assert solo.blocks(0) == (0, 1) and solo.tables(0) == (0, 1) and solo.head(0) == (0, 0)


# --- an oracle-backed stand-in for one rank's engine ---------------------------

def _header(size, address, block_type, tree_id, m0, m1, m2, cluster=CLUSTER, snapshot=SNAPSHOT_MIN):
    """Header.Block (message_header.zig:1153-1178) with the 14 metadata bytes."""
    h = np.zeros(256, np.uint8)
    h[80:96] = np.frombuffer(cluster.to_bytes(16, "little"), np.uint8)
    h[96:100] = np.frombuffer(int(size).to_bytes(4, "little"), np.uint8)
    h[110] = 20
    for off, v in ((128, m0), (132, m1), (136, m2)):
        h[off:off + 4] = np.frombuffer(int(v).to_bytes(4, "little"), np.uint8)
    h[140:142] = np.frombuffer(int(tree_id).to_bytes(2, "little"), np.uint8)
    h[224:232] = np.frombuffer(int(address).to_bytes(8, "little"), np.uint8)
    h[232:240] = np.frombuffer(int(snapshot).to_bytes(8, "little"), np.uint8)
    h[240] = block_type
    return h


def _set_checksums(block, size):
    block[32:48] = np.frombuffer(_oracle.checksum(block[256:size].tobytes()).to_bytes(16, "little"), np.uint8)
    block[0:16] = np.frombuffer(_oracle.checksum(block[16:256].tobytes()).to_bytes(16, "little"), np.uint8)


class _Buf:
    def __init__(self, eng, ptr, n):
        self.eng, self.ptr, self.nbytes = eng, ptr, n

    def download(self, n=None):
        return self.eng.mem[self.ptr:self.ptr + (self.nbytes if n is None else n)].copy()

    def free(self):
        pass


class _OracleEngine:
    """What compact_split asks of an engine, on host memory: COUNT_ONLY and
    VALUES_ONLY-at-offset merges by the oracle, copies, and tbc_compaction_seal
    restated (data_block_finish / index_block_finish from the entries)."""

    def __init__(self, spec, heap=24 << 20):
        self.mem = np.zeros(heap, np.uint8)
        self.top, self.block_size, self.spec = 4096, BS, spec
        lay = spec.layout(BS)
        self.vcm, self.dbcm = lay["block_value_count_max"], lay["data_block_count_max"]

    def layout(self, tree):
        return SimpleNamespace(block_value_count_max=self.vcm, data_block_count_max=self.dbcm)

    def alloc(self, n):
        p = self.top
        self.top += (n + 255) // 256 * 256
        assert self.top <= len(self.mem)
        return _Buf(self, p, n)

    def upload(self, a):
        b = self.alloc(a.nbytes)
        self.mem[b.ptr:b.ptr + a.nbytes] = np.frombuffer(a.tobytes(), np.uint8)
        return b

    def values(self, segs):
        vs = self.spec.value_size
        parts = [self.mem[p:p + n * vs].reshape(-1, vs) for p, n in segs]
        return np.concatenate(parts) if parts else np.zeros((0, vs), np.uint8)

    def copy_device_async(self, dst, src, n):
        self.mem[dst:dst + n] = self.mem[src:src + n].copy()

    def copy_device_batch(self, copies):
        for dst, src, n in copies:
            self.copy_device_async(dst, src, n)

    def synchronize(self):
        self.waits += 1

    def submit(self, jobs):
        from tigerbeetle_amd import abi
        (j,) = jobs
        a, b = self.values(j.segments_a), self.values(j.segments_b)
        r = _compact(_oracle, self.spec, a, j.a_immutable, b, j.drop_tombstones,
                     np.arange(1, workloads.worst_case_blocks(self.spec, max(1, len(a) + len(b)), BS) + 2,
                               dtype=np.uint64))
        surv = data_values_from_blocks(r.blocks, self.spec.value_size)
        if j.flags & abi.COMPACTION_COUNT_ONLY and j.output is not None:  # the count into a device word
            self.mem[j.output.ptr:j.output.ptr + 8] = np.frombuffer(len(surv).to_bytes(8, "little"), np.uint8)
        if j.flags & abi.COMPACTION_VALUES_ONLY:
            vs = self.spec.value_size
            for i, v in enumerate(surv):
                g = j.output_offset + i
                k = g // self.vcm
                at = j.output.ptr + split.data_block_slot(k, self.dbcm) * BS + 256 + (g - k * self.vcm) * vs
                self.mem[at:at + vs] = v
        res = SimpleNamespace(value_count=len(surv), status=0, table_count=0)
        return self._batch(res, np.zeros((0, 128), np.uint8))

    def _batch(self, res, infos):
        eng = self

        class _B:
            def wait(self):
                eng.waits += 1

            def release(self):
                pass

            def result(self, i):
                return res, infos
        return _B()

    waits = 0  # Batch.wait and synchronize calls (test_split_step_waits_once)

    def seal_submit(self, *args):
        return self._batch(*self.seal(*args))

    def seal(self, tree, cluster, snapshot_min, level_b, addresses, arena, value_count, blocks, tables):
        spec, vs, ks, vcm, dbcm = self.spec, self.spec.value_size, self.spec.key_size, self.vcm, self.dbcm
        plan = split.plan_split([value_count], vcm, dbcm)
        db = plan.data_blocks

        def slot_ptr(slot):
            return arena.ptr + slot * BS

        def key_bytes(v):
            limbs = workloads.keys_of(v[None, :], spec)
            return b"".join(int(l[0]).to_bytes(8, "little") for l in limbs).ljust(ks, b"\0")

        for k in range(*blocks):
            cnt = min(vcm, value_count - k * vcm)
            at = slot_ptr(split.data_block_slot(k, dbcm))
            blk = self.mem[at:at + BS]
            size = 256 + cnt * vs
            addr = int(addresses[split.data_block_slot(k, dbcm)])
            blk[:256] = _header(size, addr, 5, spec.tree_id, vcm, cnt, vs, cluster, snapshot_min)
            _set_checksums(blk, size)
            blk[size:-(-size // 4096) * 4096] = 0
            t, s = k // dbcm, k % dbcm
            img = slot_ptr(split.index_block_slot(t, plan.k_last(t)))
            body = blk[256:size].reshape(-1, vs)
            entry = [blk[:16].tobytes() + bytes(16), key_bytes(body[0]), key_bytes(body[-1]),
                     addr.to_bytes(8, "little")]
            for (dst, n), e in zip(split.entry_ranges(img, s, 1, dbcm, ks), entry):
                self.mem[dst:dst + n] = np.frombuffer(e, np.uint8)
        infos = []
        T = vcm * dbcm
        for t in range(*tables):
            k0, k_last = t * dbcm, plan.k_last(t)
            nblk = k_last - k0 + 1
            at = slot_ptr(split.index_block_slot(t, k_last))
            blk = self.mem[at:at + BS]
            index_size = spec.layout(BS)["index_size"]
            addr = int(addresses[split.index_block_slot(t, k_last)])
            blk[:256] = _header(index_size, addr, 4, spec.tree_id, nblk, dbcm, ks, cluster, snapshot_min)
            for dst, n in split.entry_ranges(at, nblk, dbcm - nblk, dbcm, ks):
                self.mem[dst:dst + n] = 0
            _set_checksums(blk, index_size)
            blk[index_size:-(-index_size // 4096) * 4096] = 0
            kmin = self.mem[at + 256 + 32 * dbcm: at + 256 + 32 * dbcm + ks]
            kmax_at = at + 256 + 32 * dbcm + ks * dbcm + ks * (nblk - 1)
            info = np.zeros(128, np.uint8)
            info[0:ks] = kmin
            info[32:32 + ks] = self.mem[kmax_at:kmax_at + ks]
            info[64:80] = blk[0:16]
            info[96:104] = np.frombuffer(addr.to_bytes(8, "little"), np.uint8)
            info[104:112] = np.frombuffer(int(snapshot_min).to_bytes(8, "little"), np.uint8)
            info[112:120] = 0xFF
            info[120:124] = np.frombuffer(min(T, value_count - t * T).to_bytes(4, "little"), np.uint8)
            info[124:126] = np.frombuffer(int(spec.tree_id).to_bytes(2, "little"), np.uint8)
            info[126] = (level_b & 0x3F) | (1 << 6)
            infos.append(info)
        res = SimpleNamespace(status=0, table_count=tables[1] - tables[0])
        return res, (np.stack(infos) if infos else np.zeros((0, 128), np.uint8))


class _ThreadExchange:
    """All-gathers between rank threads of one process (CPU tests)."""

    def __init__(self, world):
        self.world, self.barrier, self.slots = world, threading.Barrier(world), [None] * world

    def rank(self, r, eng):
        ex = self

        class Rank:
            """As TorchExchange over host memory (gloo): each exchange waits."""

            def count_buffer(self, engine, scratch):
                return engine.alloc(256)

            def gather_counts(self, engine, batch, buf, scratch):
                batch.wait()
                return ex._gather(r, int(batch.result(0)[0].value_count))

            def all_gather_bytes(self, engine, segments, nbytes, key, scratch):
                engine.synchronize()
                mine = b"".join(engine.mem[p:p + n].tobytes() for p, n in segments).ljust(nbytes, b"\0")
                got = ex._gather(r, mine)
                bufs = [engine.upload(np.frombuffer(g, np.uint8)) if nbytes else None for g in got]
                return bufs, [b.ptr if b else 0 for b in bufs]
        return Rank()

    def device_rank(self, r, eng):
        """As TorchExchange on the device (nccl): the count merge's word and
        the byte buffers are exchanged in stream order; the one host wait is
        reading the gathered counts (here: the count word, read once)."""
        ex = self

        class Rank:
            def count_buffer(self, engine, scratch):
                return engine.alloc(256)

            def gather_counts(self, engine, batch, buf, scratch):
                engine.waits += 1  # reading the gathered counts
                return ex._gather(r, int.from_bytes(engine.mem[buf.ptr:buf.ptr + 8].tobytes(), "little"))

            def all_gather_bytes(self, engine, segments, nbytes, key, scratch):
                mine = b"".join(engine.mem[p:p + n].tobytes() for p, n in segments).ljust(nbytes, b"\0")
                got = ex._gather(r, mine)
                bufs = [engine.upload(np.frombuffer(g, np.uint8)) if nbytes else None for g in got]
                return bufs, [b.ptr if b else 0 for b in bufs]
        return Rank()

    def _gather(self, r, x):
        self.barrier.wait()
        self.slots[r] = x
        self.barrier.wait()
        out = list(self.slots)
        self.barrier.wait()
        return out


def _run_split(spec, ji, addrs, world, cuts, exchanges, engines):
    from tigerbeetle_amd.engine import Job
    results, errors = [None] * world, []
    b_all = _b_all(ji)

    def rank(p):
        try:
            eng = engines[p]
            (a0, b0), (a1, b1) = cuts[p], cuts[p + 1]
            segs = []
            for vals in (ji.a_values[a0:a1], b_all[b0:b1]):
                buf = eng.upload(np.ascontiguousarray(vals)) if len(vals) else None
                segs.append([(buf.ptr, len(vals))] if buf else [])
            job = Job(spec, segs[0], segs[1], ji.a_immutable, ji.drop_tombstones, LEVEL_B, CLUSTER, SNAPSHOT_MIN,
                      np.asarray(addrs, np.uint64), None)
            res = split.compact_split(eng, job, cuts, exchanges[p], p, staged=True)
            eng.step_waits = eng.waits  # host waits of the enqueue (finish() waits for the rest)
            results[p] = res.finish()
        except Exception as e:  # noqa: BLE001 - reported below, other threads must not hang
            errors.append((p, repr(e)))
            exchanges[p]  # noqa: B018
            raise
    threads = [threading.Thread(target=rank, args=(p,)) for p in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not errors, errors
    return results


def _check_union(spec, ji, addrs, world, results, engines):
    whole = _compact(_oracle, spec, ji.a_values, ji.a_immutable, _b_all(ji), ji.drop_tombstones, addrs)
    plan = results[0].plan
    assert plan.total == whole.value_count
    lay = spec.layout(BS)
    vcm, dbcm = lay["block_value_count_max"], lay["data_block_count_max"]
    got = {}
    for p, res in enumerate(results):
        mem = engines[p].mem

        def block(slot):
            at = res.slot_ptr(slot)
            return mem[at:at + BS]
        for k in range(*res.blocks):
            got[split.data_block_slot(k, dbcm)] = block(split.data_block_slot(k, dbcm))
        for t in range(*res.tables):
            got[split.index_block_slot(t, plan.k_last(t))] = block(split.index_block_slot(t, plan.k_last(t)))
        # Only this rank's own slots are held: its blocks, its head block and
        # the index blocks of the tables its blocks belong to.
        lo, hi = split.slot_range(plan, p)
        assert res.arena.nbytes == (hi - lo) * BS
        assert hi - lo <= -(-plan.counts[p] // vcm) + 2 + dbcm + 1
    assert sorted(got) == list(range(len(whole.blocks)))
    for i, w in enumerate(whole.blocks):
        assert np.array_equal(disk_image(got[i]), disk_image(w)), i
    assert np.array_equal(np.concatenate([r.table_infos for r in results]), whole.table_infos)
    # Exchanged bytes: at most one partial block's values and one table's entries per rank.
    for r in results:
        assert r.exchanged["heads"] <= (vcm - 1) * spec.value_size
        assert r.exchanged["entries"] <= (dbcm - 1) * split.entry_bytes(spec.key_size)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("method", ["merge_path", "blocks"])
def test_split_job_equals_unsplit_job(oracle_lib, case, world, method):
    spec, ji, addrs = _inputs(case)
    cuts = _cuts(spec, ji, world) if method == "merge_path" else _block_cuts(spec, ji, world)
    engines = [_OracleEngine(spec) for _ in range(world)]
    tex = _ThreadExchange(world)
    results = _run_split(spec, ji, addrs, world, cuts, [tex.rank(p, engines[p]) for p in range(world)], engines)
    _check_union(spec, ji, addrs, world, results, engines)


@pytest.mark.parametrize("case", [0, 3])
@pytest.mark.parametrize("world", [2, 3])
def test_split_step_waits_once(oracle_lib, case, world):
    """With the exchange on the device (TorchExchange over nccl), a split
    step waits on the host once — for the gathered counts — and enqueues the
    rest (bodies, heads, seals, entries); over host memory (gloo) it also
    waits before each of its two byte all-gathers. Both give the unsplit
    job's bytes."""
    spec, ji, addrs = _inputs(case)
    cuts = _block_cuts(spec, ji, world)
    for device, most in ((True, 1), (False, 3)):
        engines = [_OracleEngine(spec) for _ in range(world)]
        tex = _ThreadExchange(world)
        ranks = [(tex.device_rank if device else tex.rank)(p, engines[p]) for p in range(world)]
        results = _run_split(spec, ji, addrs, world, cuts, ranks, engines)
        _check_union(spec, ji, addrs, world, results, engines)
        assert max(e.step_waits for e in engines) <= most, [e.step_waits for e in engines]


# --- the same flow with the exchange over gloo (TorchExchange), world 2 and 3 --

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
    from tigerbeetle_amd.engine import Job
    spec, ji, addrs = _inputs(case)
    reads = []
    cuts = _block_cuts(spec, ji, world, reads)      # identical on every rank, no communication
    assert len(reads) <= 2 * (world - 1)            # index keys + boundary blocks only
    eng = _OracleEngine(spec)
    (a0, b0), (a1, b1) = cuts[rank], cuts[rank + 1]
    segs = []
    for vals in (ji.a_values[a0:a1], _b_all(ji)[b0:b1]):  # stages only this rank's range
        buf = eng.upload(np.ascontiguousarray(vals)) if len(vals) else None
        segs.append([(buf.ptr, len(vals))] if buf else [])
    job = Job(spec, segs[0], segs[1], ji.a_immutable, ji.drop_tombstones, LEVEL_B, CLUSTER, SNAPSHOT_MIN,
              np.asarray(addrs, np.uint64), None)
    res = split.compact_split(eng, job, cuts, split.TorchExchange(dist), rank, staged=True).finish()
    dbcm = spec.layout(BS)["data_block_count_max"]

    def block(slot):
        at = res.slot_ptr(slot)
        return eng.mem[at:at + BS]
    mine = {split.data_block_slot(k, dbcm): bytes(disk_image(block(split.data_block_slot(k, dbcm))))
            for k in range(*res.blocks)}
    mine.update({split.index_block_slot(t, res.plan.k_last(t)):
                 bytes(disk_image(block(split.index_block_slot(t, res.plan.k_last(t))))) for t in range(*res.tables)})
    q.put((rank, mine, res.table_infos.tobytes(), res.exchanged))
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
    got = {}
    for _, mine, _, _ in out:
        got.update(mine)
    assert sorted(got) == list(range(len(whole.blocks)))
    assert [got[i] for i in range(len(whole.blocks))] == [bytes(disk_image(b)) for b in whole.blocks]
    assert b"".join(inf for _, _, inf, _ in out) == whole.table_infos.tobytes()


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
    _, ptrs = ex.all_gather_bytes(eng, [s for s in segs if s[1]], 7 * 16, "heads", {})
    got = [bytes(eng.mem.read(p, 7 * 16)) for p in ptrs]
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_bytes_host_path_over_gloo():
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
