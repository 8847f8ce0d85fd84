"""The exact benched steady state at full size.

bench.py times batches submitted back to back: up to three steps in flight
(`--depth 3`), the outputs rotating over three sets, so a step's front runs
beside the previous steps' chains and, with the chain server, every step's
chains share one ring. This drives bench.Workload through that very loop
shape (bench.run: submit, and wait for the oldest once three are pending)
and compares every job of the last three batches — blocks (disk images),
headers, TableInfos — with the oracle:

  * config 2 (BASELINE configs[1]): 28 UNIQUE_KEYS jobs per batch; the
    middle batch of the last three carries a broken speculation (one A key
    equal to a B key), so its recomputation uses the engine's mask buffer
    while the neighbouring batches' chains run;
  * config 5 (configs[4]): the throughput regime, each batch in four
    pipelined job groups.

Reference: src/lsm/compaction.zig:806-850 (block boundaries),
src/lsm/table.zig:306-457 (data/index block finish).
"""
import numpy as np
import pytest

from helpers import disk_image
from tigerbeetle_amd import configs, workloads

pytestmark = pytest.mark.gpu


def _oracle(oracle_lib, tree, a, a_immutable, b_tables, drop, level_b, bs, addrs):
    t = oracle_lib.tree(tree.tree_id, tree.key_kind, tree.usage, tree.value_size, tree.timestamp_offset,
                        tree.value_count_max, bs)
    vcm = t.block_value_count_max
    segs_a = ([a] if len(a) else []) if a_immutable else workloads.split_blocks(a, vcm)
    segs_b = [blk for tb in b_tables for blk in workloads.split_blocks(tb, vcm)]
    return oracle_lib.compact(t, segs_a, segs_b, a_immutable=a_immutable, drop_tombstones=drop, level_b=level_b,
                              cluster=0xA5A5, snapshot_min=48, addresses=addrs)


def _break_speculation(js):
    """A copy of a config-2 job's A (one disk table) with one value's id
    replaced by an id of B that sorts between its neighbours: A stays
    strictly increasing, and A and B now share a key (newest wins)."""
    a = js.a.copy()
    b0 = js.b_tables[3][1000]
    lo_b, hi_b = int(b0[0:8].view(np.uint64)[0]), int(b0[8:16].view(np.uint64)[0])
    hi, lo = a.view(np.uint64)[:, 1], a.view(np.uint64)[:, 0]  # id = hi:lo (hi most significant)
    p = int(np.searchsorted(hi, np.uint64(hi_b)))
    while p < len(a) and (int(hi[p]), int(lo[p])) < (hi_b, lo_b):
        p += 1
    assert p < len(a) - 1
    a[p, 0:16] = b0[0:16]  # the id; A's timestamp and padding stay
    return a


def _run_steady(eng, wl, job_lists, depth):
    """bench.run's loop: submit, and wait for the oldest once `depth` are
    pending; every batch is kept (not released) for the checks."""
    pending, done = [], []
    for jobs in job_lists:
        pending.append(eng.submit(jobs))
        if len(pending) >= depth:
            b = pending.pop(0)
            b.wait()
            done.append(b)
    while pending:
        b = pending.pop(0)
        b.wait()
        done.append(b)
    return done


@pytest.mark.timeout(1500)
@pytest.mark.parametrize("config", [2, 5])
def test_benched_steady_state_bit_exact(oracle_lib, config):
    import bench
    from tigerbeetle_amd import Engine, Job, abi
    from tigerbeetle_amd.engine import stage_blocks
    bs, depth = 1 << 20, 3
    job_ids = list(range(configs.DEFAULT_JOBS[config]))
    with Engine(device=0, block_size=bs, arena_bytes=2 << 30, profile=True) as eng:
        wl = bench.Workload(eng, config, job_ids, bs)
        assert wl.rotate(eng, depth) == depth
        sets = [wl.jobs] + wl.job_sets
        lists = [sets[i % depth] for i in range(2 * depth)]  # the last three batches hold the three sets
        broken = None
        if config == 2:
            # Batch 4 (set 1): job 0 with a broken speculation.
            js0 = wl.specs[0]
            a_mod = _break_speculation(js0)
            vcm = eng.layout(js0.tree).block_value_count_max
            abuf, segs_a = stage_blocks(eng, [workloads.split_blocks(a_mod, vcm)], js0.tree.value_size, bs)
            j0 = sets[1][0]
            jb = Job(js0.tree, segs_a, j0.segments_b, False, False, js0.level_b, 0xA5A5, 48, j0.addresses, j0.output,
                     flags=j0.flags)
            lists[4] = [jb] + list(sets[1][1:])
            broken = (a_mod, abuf)
        batches = _run_steady(eng, wl, lists, depth)
        try:
            # Pipelined (the chains ran beside other batches' work), as in the
            # bench's steady state; the engine picks it while a tail is running.
            piped = sum("tail_wait" in batches[bi].kernel_times() for bi in range(depth, 2 * depth))
            assert piped >= depth - 1, [batches[bi].kernel_times() for bi in range(depth, 2 * depth)]
            for bi in range(depth, 2 * depth):
                b = batches[bi]
                for i, (job, js) in enumerate(zip(lists[bi], wl.specs)):
                    a = broken[0] if (broken and bi == 4 and i == 0) else js.a
                    if js.a_unsorted:
                        t = oracle_lib.tree(js.tree.tree_id, js.tree.key_kind, js.tree.usage, js.tree.value_size,
                                            js.tree.timestamp_offset, js.tree.value_count_max, bs)
                        a = oracle_lib.sort_values(t, a)
                    o = _oracle(oracle_lib, js.tree, a, js.a_immutable, js.b_tables, js.drop_tombstones, js.level_b,
                                bs, job.addresses)
                    r, infos = b.result(i)
                    assert r.status == 0 and o.status == 0, (bi, i, r.status)
                    assert (r.value_count, r.block_count) == (o.value_count, len(o.blocks)), (bi, i)
                    if config == 2:
                        want = abi.SPECULATION_BROKEN if (bi == 4 and i == 0) else abi.SPECULATION_HELD
                        assert b.speculation(i) == want, (bi, i, b.speculation(i))
                    blocks = job.output.download(r.block_count * bs).reshape(-1, bs)
                    for k, (g, w) in enumerate(zip(blocks, o.blocks)):
                        assert np.array_equal(disk_image(g), disk_image(w)), (config, bi, i, k)
                    assert np.array_equal(infos, o.table_infos), (config, bi, i)
                    del blocks, o
                print(f"config {config} batch {bi}: {len(lists[bi])} jobs bit-exact", flush=True)
        finally:
            for b in batches:
                b.release()
