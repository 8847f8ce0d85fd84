"""GPU parity at BASELINE.json's full sizes: whole production-sized jobs of
configs 2, 3, 4 (a whole forest unit: 21 jobs of 4 key kinds in one batch)
and 5 (tigerbeetle_amd/configs.py), staged exactly as bench.py stages them (every job of the benched batch),
compared block-for-block with the oracle; plus size-independent
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


# Exactly the batches bench.py times (configs.DEFAULT_JOBS per GPU): config 2's
# 28 speculated jobs (2,016 chains at once), config 3's 28 bar-end jobs with
# their device sorts, a whole forest unit of config 4, and config 5's 27 jobs
# (13,824 output blocks: the throughput regime — 4 pipelined job groups,
# k_assemble, chain-only k_data_blocks over 1 MiB bodies).
# Configs 2-4 also through the pipelined block pass (TBC_CONFIG_PIPELINE: what
# bench.py's steps in flight take): speculated jobs merged by k_merge_unique,
# chains packed on a tail stream.
@pytest.mark.timeout(900)
@pytest.mark.parametrize("config,mode", [(2, "fused"), (2, "pipelined"), (3, "fused"), (3, "pipelined"),
                                         (4, "fused"), (4, "pipelined"), (5, "auto")])
def test_full_size_jobs_bit_exact(oracle_lib, config, mode):
    import bench
    from tigerbeetle_amd import Engine, abi
    bs = 1 << 20
    job_ids = list(range(configs.DEFAULT_JOBS[config]))
    pipeline = {"fused": False, "pipelined": True, "auto": None}[mode]
    with Engine(device=0, block_size=bs, arena_bytes=2 << 30, profile=True, pipeline=pipeline) as eng:
        wl = bench.Workload(eng, config, job_ids, bs)
        wl.step(eng).release()          # twice: the memtables are re-landed and re-sorted
        b = wl.step(eng)
        total_blocks = 0
        kernels = b.kernel_times()
        if config == 2 and mode == "fused":  # the latency regime with every job speculated (and held)
            assert "partition_blocks" in kernels and "assemble" not in kernels, kernels
        if config == 2:
            assert all(b.speculation(i) == abi.SPECULATION_HELD for i in range(len(wl.jobs)))
        if mode == "pipelined":  # speculated jobs merged tile by tile, chains on a tail
            assert "merge_unique" in kernels and "tail_wait" in kernels, kernels
        if config == 5:  # the throughput regime: pipelined groups, assembled bodies, chain-only kernel
            assert "assemble" in kernels and "tail_wait" in kernels, kernels
        for i, (job, js) in enumerate(zip(wl.jobs, wl.specs)):
            r, infos = b.result(i)
            o = _oracle_job(oracle_lib, js, bs, job.addresses)
            print(f"config {config} job {job_ids[i]}: {r.value_count} values, {r.block_count} blocks", flush=True)
            assert r.status == 0 and o.status == 0
            assert (r.value_count, r.block_count, r.table_count) == \
                (o.value_count, len(o.blocks), len(o.table_infos)), (config, job_ids[i])
            total_blocks += r.block_count
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
            del blocks, o, vals, keys
        if config == 5:
            assert total_blocks > 2 * 4096, total_blocks
        b.release()
