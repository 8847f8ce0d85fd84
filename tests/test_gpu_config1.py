"""BASELINE config 1 on the GPU: the whole `tigerbeetle benchmark` default
load (10k accounts, 10M transfers in batches of 8,190, DefaultPrng seed 42;
benchmark_load.py) committed op by op into device memtables, every bar-end
sort and every half-bar's compactions run on the GPU grid through the Forest
schedule, and each job compared byte for byte with the oracle run on the
identical inputs (LockstepExecutor): all 38 bars bench.py replays, which
include immutable flushes merging into every level-0 table they overlap,
moves of level-0 tables into level 1, and disk-A merges of a level-1 table
into the level-2 tables it overlaps. Every job must end TBC_OK
(GridExecutor.wait raises on a block error or invariant). The manifest
log's events (apply_to_manifest, remove_invisible_tables) go to blocks
closed on the GPU grid and by the oracle, compared byte for byte."""
import numpy as np
import pytest

from oracle_executor import LockstepExecutor, OracleExecutor
from tigerbeetle_amd import Grid, benchmark_load, forest
from tigerbeetle_amd.forest import GridExecutor

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_config1_all_bars_bit_exact(engine, oracle_lib):
    grid = Grid(engine, 24_000)
    try:
        lock = LockstepExecutor(GridExecutor(engine, grid), OracleExecutor(oracle_lib))
        f = forest.Forest(lock, block_count=grid.block_count, cluster=0)
        load = benchmark_load.BenchmarkLoad(transfer_count=benchmark_load.TRANSFER_COUNT)
        f.run(load.ops(), progress=lambda op: op % 32 == 0 and print(
            f"bar {op // 32}: {lock.jobs_checked} jobs, {lock.blocks_checked} blocks checked", flush=True))
        cs = [c for _, hb in f.history for _, c in hb]
        assert len(f.swaps) == 38
        assert any(c.table_a is None and c.range_b[2] for c in cs)            # immutable into overlapping L0 tables
        assert any(c.move and c.level_b == 1 for c in cs)                      # level 0 -> level 1 moves
        disk_merges = [c for c in cs if c.table_a is not None and not c.move and c.range_b[2]]
        assert disk_merges, "no disk-A merge into overlapping level-B tables"
        assert lock.jobs_checked == sum(1 for c in cs if not c.move) > 500
        # The manifest log: every event of every half-bar, blocks closed on the
        # GPU (grid) and by the oracle, byte for byte, after a checkpoint
        # closes the partial block; the log recovers the forest's tables.
        from tigerbeetle_amd import manifest
        log = f.manifest_log
        f.checkpoint_manifest()
        n_blocks = lock.manifest.check_all()
        blocks = [lock.ref.grid[a] for a in log.log_addresses]
        opened = manifest.open_log(blocks)
        want = {info.address for t in f.trees.values() for lv in t.levels for info in lv.tables}
        assert n_blocks >= 1 and set(opened) == want == set(log.table_extents)
        print(f"manifest log: {log.stats['appends']} events, {n_blocks} blocks bit-exact "
              f"({lock.manifest.compared} read back by log compaction)")
        print(f"config 1: {lock.jobs_checked} jobs ({len(disk_merges)} disk-A merges into overlapping B), "
              f"{lock.blocks_checked} blocks bit-exact over {len(f.swaps)} bars")
    finally:
        grid.close()


@pytest.mark.timeout(900)
def test_config1_checkpoint_restart_bit_exact(engine, oracle_lib):
    """The first 11 bars of the benchmark load with a checkpoint every 4 bars
    (a short vsr_checkpoint_interval): released blocks are freed at each
    checkpoint and reused by later reservations, bit-exact. Then a crash 40
    ops after the second checkpoint's trigger op and a restart from it: the
    grid's cache is cold (tbc_grid_invalidate: every block validated in full
    before use), memtables are refilled by replaying the ops after the
    checkpoint, the compactions the checkpoint holds are skipped, and the lost
    half-bars are redone with identical TableInfos. Every job is compared with
    the oracle byte for byte, before and after the restart."""
    grid = Grid(engine, 24_000)
    try:
        lock = LockstepExecutor(GridExecutor(engine, grid), OracleExecutor(oracle_lib))
        f = forest.Forest(lock, block_count=grid.block_count, cluster=0, checkpoint_interval=4 * forest.BAR)
        load = benchmark_load.BenchmarkLoad(transfer_count=11 * 32 * benchmark_load.BATCH)
        crash = 287 + 40
        f.run(load.ops(), stop=crash)
        assert [c[:2] for c in f.checkpoints] == [(127, 159), (255, 287)]
        assert f.free_set.reused > 0
        before = {op: [c.outputs for _, c in cs] for op, cs in f.history if op > 287}
        assert before
        jobs_before = lock.jobs_checked
        start = f.restart()
        assert start == 256
        n_hist = len(f.history)
        f.run(benchmark_load.BenchmarkLoad(transfer_count=11 * 32 * benchmark_load.BATCH).ops(), start=start)
        redone = {op: [c.outputs for _, c in cs] for op, cs in f.history[n_hist:] if op in before}
        assert redone == before
        assert lock.jobs_checked > jobs_before
        f.checkpoint_manifest()
        assert lock.manifest.check_all() > 0
        print(f"checkpoints {f.checkpoints}, {f.free_set.reused} reused blocks, {lock.jobs_checked} jobs bit-exact")
    finally:
        grid.close()
