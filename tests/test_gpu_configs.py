"""GPU parity at BASELINE.json's full sizes: whole production-sized jobs of
configs 2, 3, 4 (a whole forest unit: 21 jobs of 4 key kinds in one batch)
and 5 (tigerbeetle_amd/configs.py), staged exactly as bench.py stages them, compared block-for-block with the oracle; plus size-independent
properties of the output (every block's checksums verify, keys strictly
increase across the whole output, value counts add up).
"""
import numpy as np
import pytest

from helpers import disk_image
from tigerbeetle_amd import configs, workloads

pytestmark = pytest.mark.gpu


def _oracle_job(oracle_lib, js, bs, addrs):
    spec = js.tree
    t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                        spec.value_count_max, bs)
    vcm = t.block_value_count_max
    a = oracle_lib.sort_values(t, js.a) if js.a_unsorted else js.a
    segs_a = ([a] if len(a) else []) if js.a_immutable else workloads.split_blocks(a, vcm)
    segs_b = [blk for tb in js.b_tables for blk in workloads.split_blocks(tb, vcm)]
    return oracle_lib.compact(t, segs_a, segs_b, a_immutable=js.a_immutable, drop_tombstones=js.drop_tombstones,
                              level_b=js.level_b, cluster=0xA5A5, snapshot_min=48, addresses=addrs)


@pytest.mark.parametrize("config,job_ids", [(2, [0, 1]), (3, [0, 1, 6]), (4, list(range(21))), (5, [0])])
def test_full_size_jobs_bit_exact(oracle_lib, config, job_ids):
    import bench
    from tigerbeetle_amd import Engine
    bs = 1 << 20
    with Engine(device=0, block_size=bs, arena_bytes=2 << 30) as eng:
        wl = bench.Workload(eng, config, job_ids, bs)
        wl.step(eng).release()          # twice: the memtables are re-landed and re-sorted
        b = wl.step(eng)
        for i, (job, js) in enumerate(zip(wl.jobs, wl.specs)):
            r, infos = b.result(i)
            o = _oracle_job(oracle_lib, js, bs, job.addresses)
            assert r.status == 0 and o.status == 0
            assert (r.value_count, r.block_count, r.table_count) == \
                (o.value_count, len(o.blocks), len(o.table_infos)), (config, job_ids[i])
            blocks = job.output.download(r.block_count * bs).reshape(-1, bs)
            for k, (g, w) in enumerate(zip(blocks, o.blocks)):
                assert np.array_equal(disk_image(g), disk_image(w)), (config, job_ids[i], k)
            assert np.array_equal(infos, o.table_infos)
            # size-independent properties
            vs = js.tree.value_size
            data = [blk for blk in blocks if blk[240] == 5]
            assert sum(int(blk[132:136].view(np.uint32)[0]) for blk in data) == r.value_count
            vals = np.concatenate([blk[256:256 + int(blk[132:136].view(np.uint32)[0]) * vs].reshape(-1, vs)
                                   for blk in data])
            keys = np.stack(workloads.keys_of(vals, js.tree)[::-1], axis=1)
            diff = np.argmax(keys[1:] != keys[:-1], axis=1)
            rows = np.arange(len(keys) - 1)
            assert (keys[1:][rows, diff] > keys[:-1][rows, diff]).all(), "keys not strictly increasing"
            if js.drop_tombstones:
                ts = vals.view(np.uint64)[:, js.tree.timestamp_offset // 8]
                assert not (ts >> np.uint64(63)).any(), "tombstone survived the last level"
            ptrs = [job.output.ptr + k * bs + 256 for k in range(r.block_count)]
            lens = [int(blk[96:100].view(np.uint32)[0]) - 256 for blk in blocks]
            sums = eng.checksum_device(ptrs, lens)
            assert np.array_equal(sums, blocks[:, 32:48])
        b.release()
