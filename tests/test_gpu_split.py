"""Key-range split of one compaction on the GPU (tigerbeetle_amd/split.py,
SURVEY.md §8e.2): every rank runs compact_split through libtbc.so (COUNT_ONLY
merge, VALUES_ONLY at its global output offset, tbc_compaction_seal); the
data blocks, index blocks and TableInfos each rank finishes must equal, byte
for byte, the same blocks of the oracle's unsplit job, and each rank sends at
most one partial block's values and one table's index entries. Ranks share the box's one GPU (one process and engine each) and
exchange counts and heads over gloo; on an 8-GPU node the same code runs with
the nccl backend (RCCL over xGMI) and device buffers."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = {
    # 1 MiB blocks: an immutable transfers.id table into 2 level-B tables (4 output tables)
    "id_1mib": ("transfers.id", 1 << 20, None, dict(n_a=262_080, b_table_sizes=[262_080, 200_000],
                                                    a_immutable=True, dup_frac=0.02, overlap=0.3)),
    # 4 KiB blocks, small tables: many tables, heads crossing empty ranks
    "debit_4k": ("transfers.debit_account_id", 4096, 3, dict(n_a=3000, b_table_sizes=[900, 800],
                                                              a_immutable=True, dup_frac=0.2, overlap=0.2)),
    "acct_last_level_4k": ("accounts.timestamp", 4096, 3, dict(n_a=400, b_table_sizes=[200, 150],
                                                               a_immutable=False, tomb_frac=0.1,
                                                               drop_tombstones=True, overlap=0.5)),
}


def _c4_split_inputs():
    """The job bench.py splits over the ranks of config 4 at N = 2
    (SplitPart): the largest job whose A needs no device sort — a 5-table
    transfers.timestamp L1->L2 compaction, 168 MB — with bench's addresses."""
    from tigerbeetle_amd import configs, workloads
    bs = 1 << 20
    ids = [j for j in range(2 * configs.DEFAULT_JOBS[4]) if configs.presorted(4, j)]
    gid = max(ids, key=lambda j: configs.job_bytes(4, j))
    js = configs.GENERATORS[4](gid)
    assert not js.a_unsorted
    ji = workloads.JobInputs(js.tree, js.a, js.a_immutable, list(js.b_tables), js.drop_tombstones)
    dbcm = js.tree.layout(bs)["data_block_count_max"]
    reservation = (len(js.b_tables) + 1) * dbcm + len(js.b_tables) + 1
    return js.tree, bs, ji, np.arange(1, reservation + 1, dtype=np.uint64)


def _inputs(name):
    from tigerbeetle_amd import trees, workloads
    if name == "c4_split":
        return _c4_split_inputs()
    tree, bs, tables, kw = CASES[name]
    spec = trees.BY_NAME[tree]
    if tables:
        spec = trees.with_table_size(spec, tables * (bs - 256) // spec.value_size + 5)
    rng = np.random.default_rng(sum(map(ord, name)))
    ji = workloads.make_job_inputs(spec, rng, **kw)
    n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n, bs) + 2, rng, 77, 0.05)
    return spec, bs, ji, addrs


def _run_rank(name, rank, world, exchange, max_engine_waits=None):
    """compact_split on this rank; returns (ok, message). With
    max_engine_waits, the engine-level host waits (Batch.wait, synchronize,
    downloads) made while compact_split enqueues the step must not exceed it."""
    from helpers import disk_image, run_oracle
    from oracle import oracle
    from tigerbeetle_amd import Engine, split, workloads
    from tigerbeetle_amd.engine import Job, stage_blocks
    spec, bs, ji, addrs = _inputs(name)
    with Engine(device=0, block_size=bs) as eng:
        lay = eng.layout(spec)
        vcm, dbcm = lay.block_value_count_max, lay.data_block_count_max
        # Splitters from the inputs' data-block first keys (index blocks),
        # cuts from one boundary block per side; then this rank stages only
        # its own range of A and of B (per-rank staging).
        b_all = np.concatenate(ji.b_tables)
        side_a = split.BlockedSide.from_values(workloads.keys_of(ji.a_values, spec), len(ji.a_values), vcm)
        side_b = split.BlockedSide.from_values(workloads.keys_of(b_all, spec), len(b_all), vcm)
        cuts = split.block_cuts(side_a, side_b, split.block_splitters(side_a, side_b, world))
        (a0, b0), (a1, b1) = cuts[rank], cuts[rank + 1]
        a_mine, b_mine = ji.a_values[a0:a1], b_all[b0:b1]
        if ji.a_immutable:
            abuf = eng.upload(a_mine) if len(a_mine) else None
            segs_a = [(abuf.ptr, len(a_mine))] if abuf else []
        else:
            abuf, segs_a = stage_blocks(eng, [workloads.split_blocks(a_mine, vcm)], spec.value_size, bs)
        bbuf, segs_b = stage_blocks(eng, [workloads.split_blocks(b_mine, vcm)], spec.value_size, bs)
        assert split.staged_bytes(cuts, rank, spec.value_size) == a_mine.nbytes + b_mine.nbytes
        job = Job(spec, segs_a, segs_b, ji.a_immutable, ji.drop_tombstones, 1, 0x1234, 48,
                  np.asarray(addrs, dtype=np.uint64), None)
        waits = _count_engine_waits() if max_engine_waits is not None else None
        try:
            res = split.compact_split(eng, job, cuts, exchange, rank, staged=True)
        finally:
            n_waits = waits() if waits else 0
        if max_engine_waits is not None and n_waits > max_engine_waits:
            return False, f"rank {rank}: {n_waits} engine waits while enqueuing the step"
        res = res.finish()
        whole = run_oracle(oracle, ji, bs, addrs)
        assert whole.status == 0
        plan = res.plan
        if plan.total != whole.value_count:
            return False, f"rank {rank}: total {plan.total} != {whole.value_count}"
        if res.exchanged["heads"] > (vcm - 1) * spec.value_size or \
                res.exchanged["entries"] > (dbcm - 1) * split.entry_bytes(spec.key_size):
            return False, f"rank {rank}: exchanged {res.exchanged}"
        got = res.arena.download().reshape(-1, bs)  # this rank's slots only (split.slot_range)
        slots = [split.data_block_slot(k, dbcm) for k in range(*res.blocks)]
        slots += [split.index_block_slot(t, plan.k_last(t)) for t in range(*res.tables)]
        for slot in slots:
            if not np.array_equal(disk_image(got[slot - res.base_slot]), disk_image(whole.blocks[slot])):
                return False, f"rank {rank}: block slot {slot} differs"
        t0, t1 = res.tables
        if not np.array_equal(res.table_infos, whole.table_infos[t0:t1]):
            return False, f"rank {rank}: TableInfo differs"
        return True, f"rank {rank}: blocks {res.blocks} tables {res.tables} OK ({len(slots)} slots)"


_WAITS = None


def _count_engine_waits():
    """Count this thread's engine host waits (Batch.wait, synchronize,
    downloads) from now on; returns a function that stops counting and gives
    the count. The methods are wrapped once per process; each thread counts
    only its own calls (ranks may be threads of one process)."""
    import threading
    from tigerbeetle_amd import engine as E
    global _WAITS
    if _WAITS is None:
        _WAITS = threading.local()
        for cls, m in ((E.Batch, "wait"), (E.Engine, "synchronize"), (E.DeviceBuffer, "download")):
            f = getattr(cls, m)

            def counted(*a, _f=f, **k):
                if getattr(_WAITS, "on", False):
                    _WAITS.n += 1
                return _f(*a, **k)
            setattr(cls, m, counted)
    _WAITS.on, _WAITS.n = True, 0

    def stop():
        _WAITS.on = False
        return _WAITS.n
    return stop


def test_split_single_rank_bit_exact():
    from tigerbeetle_amd import split
    ok, msg = _run_rank("debit_4k", 0, 1, split.SingleRank())
    assert ok, msg


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(name, rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tigerbeetle_amd import split
    try:
        q.put(_run_rank(name, rank, world, split.TorchExchange(dist)))
    except Exception as e:  # report, do not hang the other ranks' queue reads
        q.put((False, f"rank {rank}: {type(e).__name__}: {e}"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("id_1mib", 2), ("debit_4k", 3), ("acct_last_level_4k", 4),
                                        ("c4_split", 2)])  # the job bench splits, full size
def test_split_ranks_bit_exact(name, world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(name, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert all(ok for ok, _ in out), [m for _, m in out]
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("bs,name", [(4096, "debit_4k"), (1 << 20, "id_1mib")])
def test_values_only_bodies_equal_full_compaction(bs, name):
    """TBC_COMPACTION_VALUES_ONLY (split phase 1): the data-block bodies and
    result counts of a full compaction; headers, checksums and index blocks
    are not written."""
    from helpers import gpu_run
    from tigerbeetle_amd import Engine, abi, split
    from tigerbeetle_amd.engine import Job, stage_blocks
    from tigerbeetle_amd import workloads
    spec, bs, ji, addrs = _inputs(name)
    with Engine(device=0, block_size=bs) as eng:
        (full, _, blocks), = gpu_run(eng, [ji], bs, [addrs])[0]
        lay = eng.layout(spec)
        vcm, dbcm = lay.block_value_count_max, lay.data_block_count_max
        abuf = eng.upload(ji.a_values)
        bbuf, segs_b = stage_blocks(eng, [workloads.split_blocks(t, vcm) for t in ji.b_tables], spec.value_size, bs)
        out = eng.alloc(len(addrs) * bs)
        out.zero()
        job = Job(spec, [(abuf.ptr, len(ji.a_values))], segs_b, True, ji.drop_tombstones, 1, 0x1234, 48,
                  np.asarray(addrs, dtype=np.uint64), out, flags=abi.COMPACTION_VALUES_ONLY)
        b = eng.submit([job])
        b.wait()
        r, infos = b.result(0)
        b.release()
        assert (r.status, r.value_count, r.data_block_count, r.table_count) == \
            (0, full.value_count, full.data_block_count, full.table_count)
        got = out.download(full.block_count * bs).reshape(-1, bs)
        vs = spec.value_size
        for k in range(full.data_block_count):
            slot = k + k // dbcm
            n = min(vcm, full.value_count - k * vcm)
            assert np.array_equal(got[slot, 256:256 + n * vs], blocks[slot, 256:256 + n * vs]), k
            assert not got[slot, :256].any()
        for t in range(full.table_count):
            assert not got[min((t + 1) * (dbcm + 1), full.block_count) - 1].any()
        # mixed flags in one batch are refused
        job2 = Job(spec, [(abuf.ptr, len(ji.a_values))], segs_b, True, ji.drop_tombstones, 1, 0x1234, 48,
                   np.asarray(addrs, dtype=np.uint64), out)
        with pytest.raises(Exception):
            eng.submit([job, job2])


@pytest.mark.parametrize("bs,name", [(4096, "debit_4k"), (1 << 20, "id_1mib")])
def test_count_only_and_values_at_offset(bs, name):
    """TBC_COMPACTION_COUNT_ONLY gives the full compaction's survivor count and
    writes nothing; VALUES_ONLY with output_offset places survivor i at the
    job's output position offset + i (block and slot of the job's layout)."""
    from helpers import gpu_run
    from tigerbeetle_amd import Engine, abi, split
    from tigerbeetle_amd.engine import Job, stage_blocks
    from tigerbeetle_amd import workloads
    spec, bs, ji, addrs = _inputs(name)
    with Engine(device=0, block_size=bs) as eng:
        (full, _, blocks), = gpu_run(eng, [ji], bs, [addrs])[0]
        lay = eng.layout(spec)
        vcm, dbcm, vs = lay.block_value_count_max, lay.data_block_count_max, spec.value_size
        abuf = eng.upload(ji.a_values)
        bbuf, segs_b = stage_blocks(eng, [workloads.split_blocks(t, vcm) for t in ji.b_tables], vs, bs)
        a_seg = [(abuf.ptr, len(ji.a_values))]
        cnt = Job(spec, a_seg, segs_b, True, ji.drop_tombstones, 1, 0x1234, 48, np.zeros(0, np.uint64), None,
                  flags=abi.COMPACTION_COUNT_ONLY)
        b = eng.submit([cnt])
        b.wait()
        r, _ = b.result(0)
        b.release()
        assert r.status == 0 and r.value_count == full.value_count
        off = vcm // 3 + 7  # not a block boundary
        n_in = len(ji.a_values) + sum(len(t) for t in ji.b_tables)  # the engine bounds the range by its inputs
        n_slots = split.data_block_slot((off + n_in - 1) // vcm, dbcm) + 1
        out = eng.alloc(n_slots * bs)
        out.zero()
        job = Job(spec, a_seg, segs_b, True, ji.drop_tombstones, 1, 0x1234, 48,
                  np.arange(1, n_slots + 1, dtype=np.uint64), out, flags=abi.COMPACTION_VALUES_ONLY,
                  output_offset=off)
        b = eng.submit([job])
        b.wait()
        r, _ = b.result(0)
        b.release()
        assert r.status == 0 and r.value_count == full.value_count
        got = out.download().reshape(-1, bs)
        placed = []
        for g in range(off, off + full.value_count, 1):
            k = g // vcm
            if g == off or g % vcm == 0:
                end = min((k + 1) * vcm, off + full.value_count)
                row = got[split.data_block_slot(k, dbcm)]
                placed.append(row[256 + (g - k * vcm) * vs: 256 + (end - k * vcm) * vs].reshape(-1, vs))
        want = np.concatenate([blocks[split.data_block_slot(k, dbcm), 256:256 + min(vcm, full.value_count - k * vcm)
                                      * vs].reshape(-1, vs) for k in range(full.data_block_count)])
        assert np.array_equal(np.concatenate(placed), want)


# ---------------------------------------------------------------------------
# The device exchange (TorchExchange on a cuda device: the count word, the
# all-gathers on the engine stream through torch.cuda.ExternalStream), which
# bench.py takes at N > 1 with the nccl backend.

def _nccl_worker(names, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("nccl", rank=0, world_size=1)  # RCCL, before any other GPU work
    from tigerbeetle_amd import split
    try:
        out = []
        for name in names:
            ex = split.TorchExchange(dist, "cuda:0")
            assert ex.on_device
            # The step's one host wait is reading the gathered counts (a
            # torch copy); the engine itself is not waited for.
            out.append(_run_rank(name, 0, 1, ex, max_engine_waits=0))
        q.put((all(ok for ok, _ in out), [m for _, m in out]))
    except Exception as e:
        q.put((False, f"{type(e).__name__}: {e}"))
    dist.destroy_process_group()


def test_split_over_rccl_world_one_bit_exact():
    """The nccl (RCCL) branch of the split exchange executed: a world of one
    (RCCL refuses two ranks on one device, and the pool's boxes have one
    GPU), so only the counts all-gather runs — on the engine stream, over
    the device count word — for config 4's split job and a 4 KiB case; the
    blocks and TableInfos equal the oracle's unsplit job."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(["c4_split", "debit_4k"], _free_port(), q))
    p.start()
    ok, msg = q.get(timeout=300)
    p.join(timeout=60)
    if p.is_alive():
        p.kill()
    assert ok, msg
    assert p.exitcode == 0


class _StreamDist:
    """A torch.distributed stand-in for ranks that are threads of one
    process on one GPU, for TorchExchange's device branch. Like RCCL's
    collective, all_gather_into_tensor is ordered on each rank's CURRENT
    stream (the engine stream the exchange put in front): each rank records
    an event where its input is ready, and after a thread barrier every rank
    waits (on its stream) for every rank's event and copies every rank's
    input into its output on that stream; a second round keeps any rank from
    reusing its input before all ranks have copied it."""

    def __init__(self, world):
        import threading
        self.world = world
        self.barrier = threading.Barrier(world)
        self.local = threading.local()
        self.inputs = [None] * world
        self.copied = [None] * world
        self.calls = 0

    def get_rank(self):
        return self.local.rank

    def get_world_size(self):
        return self.world

    def all_gather_into_tensor(self, out, inp):
        import torch
        r, s = self.local.rank, torch.cuda.current_stream()
        ready = torch.cuda.Event()
        ready.record(s)
        self.inputs[r] = (inp, ready)
        self.barrier.wait()
        n = inp.numel()
        for q, (t, ev) in enumerate(self.inputs):
            s.wait_event(ev)
            out[q * n:(q + 1) * n].copy_(t)
        done = torch.cuda.Event()
        done.record(s)
        self.copied[r] = done
        self.barrier.wait()
        for ev in self.copied:
            s.wait_event(ev)
        if r == 0:
            self.calls += 1
        self.barrier.wait()


@pytest.mark.parametrize("name,world", [("debit_4k", 2), ("id_1mib", 2), ("c4_split", 2)])
def test_split_device_exchange_stream_order(name, world):
    """TorchExchange's device branch end to end on the real engine: `world`
    ranks as threads of this process, one Engine each on cuda:0, exchanging
    through _StreamDist on their engine streams — the count word, the heads'
    and the index entries' all-gathers and the copies into place, all in
    engine-stream order with no engine wait while the step is enqueued. Every
    rank's blocks and TableInfos equal the oracle's unsplit job."""
    import threading
    from tigerbeetle_amd import split
    d = _StreamDist(world)
    results = [None] * world
    _count_engine_waits()()  # wrap the wait methods once, before the rank threads start

    def run(r):
        d.local.rank = r
        try:
            results[r] = _run_rank(name, r, world, split.TorchExchange(d, "cuda:0"), max_engine_waits=0)
        except Exception as e:  # noqa: BLE001 - reported below
            results[r] = (False, f"rank {r}: {type(e).__name__}: {e}")
            d.barrier.abort()

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert all(res is not None and res[0] for res in results), results
    # the counts, and (a straddling block: its heads) at 1 MiB blocks
    assert d.calls >= (2 if name == "id_1mib" else 1), d.calls
