"""Throughput-regime chains in the column-pair layout (aegis.hip
k_data_blocks_col2: four blocks per wave, 16 lanes per message; waves with a
partial block fall back to two pairs of the 32-lane layout).

Batches with more than 4,096 output blocks (4 KiB blocks keep them small):
one job (plain throughput regime, launch_blocks) and two jobs (job groups,
chains on the tail streams, launch_blocks_tail), accounts.timestamp with
last-level tombstone drops and overlapping keys (config 5's shape), compared
block-for-block with the oracle.
"""
import numpy as np
import pytest

from helpers import disk_image, gpu_run, run_oracle
from tigerbeetle_amd import trees, workloads

pytestmark = pytest.mark.gpu

BS = 4096


def _spec():
    base = trees.BY_NAME["accounts.timestamp"]
    return trees.with_table_size(base, 5 * (BS - 256) // base.value_size + 3)


def _case(rng, n_a, n_tables):
    spec = _spec()
    per = spec.value_count_max
    ji = workloads.make_job_inputs(spec, rng, n_a=n_a, b_table_sizes=[per] * n_tables, a_immutable=False,
                                   overlap=0.3, tomb_frac=0.05, drop_tombstones=True)
    n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n, BS) + 3, rng, int(rng.integers(1, 1000)), 0.1)
    return ji, addrs


def _check(oracle_lib, inputs, addrs, results):
    for ji, a, (r, infos, blocks) in zip(inputs, addrs, results):
        o = run_oracle(oracle_lib, ji, BS, a)
        assert r.status == 0 and o.status == 0
        assert r.block_count == len(o.blocks) and r.value_count == o.value_count
        for g, w in zip(blocks, o.blocks):
            assert np.array_equal(disk_image(g), disk_image(w))
        assert np.array_equal(infos, o.table_infos)


def test_col2_single_job(oracle_lib, engine_small):
    rng = np.random.default_rng(55)
    ji, a = _case(rng, 40_000, 640)   # ~4,400 output blocks: > 2,048 chain waves
    results, _ = gpu_run(engine_small, [ji], BS, [a])
    assert results[0][0].data_block_count > 4096
    _check(oracle_lib, [ji], [a], results)


def test_col2_job_groups(oracle_lib, engine_small):
    rng = np.random.default_rng(56)
    cases = [_case(rng, 40_000, 640), _case(rng, 38_000, 650)]
    inputs, addrs = [c[0] for c in cases], [c[1] for c in cases]
    results, _ = gpu_run(engine_small, inputs, BS, addrs)
    _check(oracle_lib, inputs, addrs, results)
