"""Batches submitted back to back without waiting (as bench.py's timed loop
does): the second batch writes the same caller-provided output blocks the
first one's tail streams (chains, in the throughput regime's pipelined
groups) may still be reading, so its fronts must start after those tails
(engine.hip tbc_compaction_submit). The outputs must end as the oracle's
compaction of the SECOND batch's inputs, headers included."""
import numpy as np
import pytest

from helpers import disk_image, run_oracle
from tigerbeetle_amd import trees, workloads
from tigerbeetle_amd.engine import Job, stage_blocks

BS = 4096


def _cases():
    T = trees.BY_NAME
    cases = []
    for i, name in enumerate(["transfers.id", "accounts.timestamp", "transfers.debit_account_id", "accounts.ledger",
                              "posted.timestamp", "transfers.id", "account_history.timestamp", "transfers.amount"]):
        base = T[name]
        spec = trees.with_table_size(base, 6 * (BS - 256) // base.value_size + 1)
        n = 125 * (BS - 256) // base.value_size
        cases.append((spec, dict(n_a=n, b_table_sizes=[n // 2] * 7, a_immutable=i % 2 == 1, dup_frac=0.1 * (i % 2),
                                 tomb_frac=0.05 * (i % 3 != 2), drop_tombstones=i % 4 == 3, overlap=0.2)))
    return cases


def _jobs(engine, inputs, addrs, outs, keep, bs=BS, flags=0):
    jobs = []
    for ji, a, out in zip(inputs, addrs, outs):
        vcm = engine.layout(ji.tree).block_value_count_max
        if ji.a_immutable:
            abuf = engine.upload(ji.a_values)
            segs_a = [(abuf.ptr, len(ji.a_values))]
        else:
            abuf, segs_a = stage_blocks(engine, [workloads.split_blocks(ji.a_values, vcm)], ji.tree.value_size, bs)
        bbuf, segs_b = stage_blocks(engine, [workloads.split_blocks(t, vcm) for t in ji.b_tables],
                                    ji.tree.value_size, bs)
        keep += [abuf, bbuf]
        jobs.append(Job(ji.tree, segs_a, segs_b, ji.a_immutable, ji.drop_tombstones, 1, 0x1234, 48, a, out,
                        flags=flags))
    return jobs


@pytest.mark.gpu
def test_back_to_back_batches_share_outputs(engine_small, oracle_lib):
    cases = _cases()
    rng1, rng2, rng_a = np.random.default_rng(301), np.random.default_rng(302), np.random.default_rng(303)
    first = [workloads.make_job_inputs(spec, rng1, **kw) for spec, kw in cases]
    second = [workloads.make_job_inputs(spec, rng2, **kw) for spec, kw in cases]
    addrs, outs = [], []
    for (spec, kw), ji in zip(cases, first):
        n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
        a = workloads.addresses_for(workloads.worst_case_blocks(spec, 2 * n, BS) + 3, rng_a, 1, 0.1)
        addrs.append(np.asarray(a, dtype=np.uint64))
        out = engine_small.alloc(len(a) * BS)
        out.zero()
        outs.append(out)
    assert sum(workloads.worst_case_blocks(s, kw["n_a"] * 9 // 2, BS) for s, kw in cases) > 4096  # pipelined groups
    keep = []
    b1 = engine_small.submit(_jobs(engine_small, first, addrs, outs, keep))
    b2 = engine_small.submit(_jobs(engine_small, second, addrs, outs, keep))
    b1.wait()
    b2.wait()
    for i, (ji, a, out) in enumerate(zip(second, addrs, outs)):
        r, infos = b2.result(i)
        o = run_oracle(oracle_lib, ji, BS, a)
        assert r.status == 0 and o.status == 0
        assert r.block_count == len(o.blocks)
        got = out.download(r.block_count * BS).reshape(-1, BS)
        for k, (g, w) in enumerate(zip(got, o.blocks)):
            assert np.array_equal(disk_image(g), disk_image(w)), (ji.tree.name, k)
        assert np.array_equal(infos, o.table_infos)
    b1.release()
    b2.release()


@pytest.mark.gpu
def test_back_to_back_speculated_batches_share_outputs(engine, oracle_lib):
    """The latency regime: a UNIQUE_KEYS batch's index blocks and results run
    on a tail stream; a second batch into the same output blocks must wait
    for them (its data blocks, then its own index blocks, are the final ones)."""
    from tigerbeetle_amd import abi
    bs = 1 << 20
    names = ["transfers.id", "transfers.timestamp", "transfers.debit_account_id", "transfers.amount"]
    rng1, rng2, rng_a = np.random.default_rng(311), np.random.default_rng(312), np.random.default_rng(313)
    kw = dict(n_a=60_000, b_table_sizes=[50_000, 40_000], a_immutable=False, overlap=0.3)
    first = [workloads.make_job_inputs(trees.BY_NAME[n], rng1, **kw) for n in names]
    second = [workloads.make_job_inputs(trees.BY_NAME[n], rng2, **kw) for n in names]
    addrs, outs = [], []
    for n in names:
        a = workloads.addresses_for(workloads.worst_case_blocks(trees.BY_NAME[n], 150_000, bs) + 3, rng_a, 1, 0.1)
        addrs.append(np.asarray(a, dtype=np.uint64))
        out = engine.alloc(len(a) * bs)
        out.zero()
        outs.append(out)
    keep = []
    fl = abi.COMPACTION_UNIQUE_KEYS
    j1, j2 = _jobs(engine, first, addrs, outs, keep, bs, fl), _jobs(engine, second, addrs, outs, keep, bs, fl)
    b1 = engine.submit(j1)
    b2 = engine.submit(j2)
    b1.wait()
    b2.wait()
    for i, (ji, a, out) in enumerate(zip(second, addrs, outs)):
        r, infos = b2.result(i)
        o = run_oracle(oracle_lib, ji, bs, a)
        assert r.status == 0 and o.status == 0
        assert r.block_count == len(o.blocks)
        got = out.download(r.block_count * bs).reshape(-1, bs)
        for k, (g, w) in enumerate(zip(got, o.blocks)):
            assert np.array_equal(disk_image(g), disk_image(w)), (ji.tree.name, k)
        assert np.array_equal(infos, o.table_infos)
    b1.release()
    b2.release()


@pytest.mark.gpu
def test_speculated_batches_pipelined_three_in_flight(engine, oracle_lib):
    """Round 4: a UNIQUE_KEYS batch submitted while an earlier batch's tail is
    running is pipelined (bodies merged by k_merge_unique on the engine
    stream, chains on a tail stream beside the earlier batches' chains).
    Three batches into three output sets, then a fourth into the first set
    (it must wait for the first batch's tail), submitted without waiting;
    held and broken speculations mixed. Every batch's TableInfos and the
    final blocks of every output set equal the oracle's."""
    from tigerbeetle_amd import abi
    bs = 1 << 20
    names = ["transfers.id", "transfers.timestamp", "transfers.debit_account_id", "transfers.amount"]
    rng_a = np.random.default_rng(413)
    kw = dict(n_a=60_000, b_table_sizes=[50_000, 40_000], a_immutable=False, overlap=0.0)
    kw_broken = dict(kw, overlap=0.01)
    inputs = []
    for step in range(4):
        rng = np.random.default_rng(400 + step)
        inputs.append([workloads.make_job_inputs(trees.BY_NAME[n], rng, **(kw_broken if (step + i) % 3 == 0 else kw))
                       for i, n in enumerate(names)])
    addrs = [np.asarray(workloads.addresses_for(workloads.worst_case_blocks(trees.BY_NAME[n], 150_000, bs) + 3,
                                                rng_a, 1, 0.1), dtype=np.uint64) for n in names]
    sets = []
    for _ in range(3):
        outs = []
        for a in addrs:
            out = engine.alloc(len(a) * bs)
            out.zero()
            outs.append(out)
        sets.append(outs)
    keep = []
    fl = abi.COMPACTION_UNIQUE_KEYS
    job_lists = [_jobs(engine, inputs[s], addrs, sets[s % 3], keep, bs, fl) for s in range(4)]  # staged first
    batches = [engine.submit(jl) for jl in job_lists]  # back to back: earlier tails still running
    for b in batches:
        b.wait()
    for s, b in enumerate(batches):
        if s:  # submitted while an earlier batch's tail ran: the pipelined pass
            assert "merge_unique" in b.kernel_times(), s
        for i, ji in enumerate(inputs[s]):
            r, infos = b.result(i)
            o = run_oracle(oracle_lib, ji, bs, addrs[i])
            assert r.status == 0 and o.status == 0
            assert r.block_count == len(o.blocks) and np.array_equal(infos, o.table_infos), (s, i)
            if s >= 1:  # set 0's blocks are batch 3's (batch 0's were overwritten)
                got = sets[s % 3][i].download(r.block_count * bs).reshape(-1, bs)
                for k, (g, w) in enumerate(zip(got, o.blocks)):
                    assert np.array_equal(disk_image(g), disk_image(w)), (s, ji.tree.name, k)
    for b in batches:
        b.release()


@pytest.mark.gpu
def test_early_prep_waits_for_engine_stream_writes(engine_pipe, oracle_lib):
    """a pipelined speculated batch uploads its descriptors
    and runs its merge-path partition ahead on a tail stream, off the engine
    stream. Its inputs here are all still being written on the engine stream
    when it is submitted — A put into a device memtable in random order and
    sorted out of place (tbc_memtable_put, tbc_sort_values_batch), B landed
    by a device copy (tbc_copy_device_batch) — with no host wait in between;
    the partition must see the final bytes: blocks and TableInfos equal the
    oracle's, twice (the second batch also overlaps the first one's tail)."""
    from tigerbeetle_amd import Memtable, abi
    from tigerbeetle_amd.engine import Job
    bs = 1 << 20
    eng = engine_pipe
    spec = trees.BY_NAME["transfers.id"]
    vcm = eng.layout(spec).block_value_count_max
    rng = np.random.default_rng(521)
    batches, keep = [], []
    for step in range(2):
        ji = workloads.make_job_inputs(spec, rng, n_a=spec.value_count_max, b_table_sizes=[8 * vcm, 8 * vcm],
                                       a_immutable=True, overlap=0.0)
        addrs = np.arange(1, workloads.worst_case_blocks(spec, 3 * spec.value_count_max, bs) + 3, dtype=np.uint64)
        out = eng.alloc(len(addrs) * bs)
        mem = Memtable(eng, spec)
        a_sorted = eng.alloc(ji.a_values.nbytes)
        b_host = np.concatenate(ji.b_tables)
        b_src = eng.upload(b_host)  # synchronous: before any of the writes below
        b_dst = eng.alloc(b_host.nbytes)
        keep += [out, mem, a_sorted, b_src, b_dst]
        eng.synchronize()
        # Enqueued on the engine stream, no host wait from here to the submit.
        mem.put(ji.a_values[rng.permutation(len(ji.a_values))])
        ptr, n = mem.values()
        eng.sort_values_batch([(spec, ptr, n, a_sorted.ptr)])
        eng.copy_device_batch([(b_dst.ptr, b_src.ptr, b_host.nbytes)])
        segs_b = [(b_dst.ptr + o * spec.value_size, len(t)) for o, t in
                  zip(np.cumsum([0] + [len(t) for t in ji.b_tables[:-1]]), ji.b_tables)]
        job = Job(spec, [(a_sorted.ptr, n)], segs_b, True, False, 1, 0x1234, 48, addrs, out,
                  flags=abi.COMPACTION_UNIQUE_KEYS)
        batches.append((eng.submit([job]), ji, addrs, out, job))
    for b, ji, addrs, out, _ in batches:
        b.wait()
        assert "merge_unique" in b.kernel_times()  # the pipelined pass (TBC_CONFIG_PIPELINE)
        r, infos = b.result(0)
        o = run_oracle(oracle_lib, ji, bs, addrs)
        assert r.status == 0 and o.status == 0 and r.block_count == len(o.blocks)
        got = out.download(r.block_count * bs).reshape(-1, bs)
        for k, (g, w) in enumerate(zip(got, o.blocks)):
            assert np.array_equal(disk_image(g), disk_image(w)), k
        assert np.array_equal(infos, o.table_infos)
        b.release()
    for m in keep:
        if hasattr(m, "close"):
            m.close()


@pytest.mark.gpu
def test_engine_closed_with_live_batches_then_a_new_engine(oracle_lib):
    """an engine closed while batches are still in flight
    (never waited for, never released) leaves no HIP error behind: a second
    engine's compaction afterwards is bit-exact, and its calls report no
    stale error (tbc returns TBC_ERR_DEVICE for an unreported one)."""
    from helpers import gpu_run
    from tigerbeetle_amd import Engine, abi
    bs = 1 << 20
    spec = trees.BY_NAME["transfers.id"]
    rng = np.random.default_rng(77)
    ji = workloads.make_job_inputs(spec, rng, n_a=200_000, b_table_sizes=[150_000, 100_000], a_immutable=True,
                                   overlap=0.0)
    addrs = np.arange(1, workloads.worst_case_blocks(spec, 450_000, bs) + 3, dtype=np.uint64)
    e1 = Engine(device=0, block_size=bs)
    keep = []
    live = []
    for _ in range(3):
        live.append(e1.submit(_jobs(e1, [ji], [addrs], [e1.alloc(len(addrs) * bs)], keep, bs,
                                    abi.COMPACTION_UNIQUE_KEYS)))
    e1.close()  # batches still in flight: their handles die with the engine
    with Engine(device=0, block_size=bs) as e2:
        (r, infos, blocks), = gpu_run(e2, [ji], bs, [addrs], flags=abi.COMPACTION_UNIQUE_KEYS)[0]
        o = run_oracle(oracle_lib, ji, bs, addrs)
        assert r.status == 0 and r.block_count == len(o.blocks)
        for g, w in zip(blocks, o.blocks):
            assert np.array_equal(disk_image(g), disk_image(w))
        assert np.array_equal(infos, o.table_infos)
        e2.synchronize()
    del live
