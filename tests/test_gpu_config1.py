"""BASELINE config 1 on the GPU: the `tigerbeetle benchmark` default load
(10k accounts, transfers in batches of 8,190, DefaultPrng seed 42;
benchmark_load.py) committed op by op into device memtables, the bar-end
sorts and every half-bar's compactions run on the GPU grid through the
Forest schedule, and each job compared byte for byte with the oracle run on
the identical inputs (LockstepExecutor): the first 11 bars, which include
immutable flushes merging into every level-0 table they overlap, and moves
of level-0 tables into level 1."""
import numpy as np
import pytest

from oracle_executor import LockstepExecutor, OracleExecutor
from tigerbeetle_amd import Grid, benchmark_load, forest
from tigerbeetle_amd.forest import GridExecutor

pytestmark = pytest.mark.gpu

BARS = 11


def test_config1_first_bars_bit_exact(engine, oracle_lib):
    grid = Grid(engine, 12_000)
    try:
        lock = LockstepExecutor(GridExecutor(engine, grid), OracleExecutor(oracle_lib))
        f = forest.Forest(lock, block_count=grid.block_count, cluster=0)
        load = benchmark_load.BenchmarkLoad(transfer_count=BARS * 32 * benchmark_load.BATCH)
        f.run(load.ops(), progress=lambda op: op % 32 == 0 and print(f"bar {op // 32}: {lock.jobs_checked} jobs checked", flush=True))
        kinds = {(c.table_a is None, c.move, c.level_b) for _, cs in f.history for _, c in cs}
        assert (True, False, 0) in kinds              # immutable -> level 0
        assert (False, True, 1) in kinds              # level 0 -> level 1 moves
        assert lock.jobs_checked > 100 and lock.blocks_checked > 1000
        print(f"config 1: {lock.jobs_checked} jobs, {lock.blocks_checked} blocks bit-exact over {BARS} bars")
    finally:
        grid.close()
