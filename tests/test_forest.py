"""CPU tests of the host-side replay of BASELINE config 1 (no GPU): the
benchmark load generator (benchmark_load.zig restated), the FreeSet and
Manifest restatements, and a small `tigerbeetle benchmark` replay through
the Forest schedule with the oracle as the executor."""
import numpy as np

from oracle_executor import OracleExecutor
from tigerbeetle_amd import benchmark_load, forest, trees, workloads
from tigerbeetle_amd.tables import SNAPSHOT_LATEST, TableInfo


def test_table_count_max_for_level():
    # tree.zig:1121-1138
    assert [forest.table_count_max_for_level(l) for l in range(3)] == [8, 64, 512]


def test_free_set_reservations_are_disjoint_windows_of_free_blocks():
    fs = forest.FreeSet(64)
    fs.acquire(np.array([2, 3, 7], dtype=np.uint64))
    r1 = fs.reserve(4)              # blocks 0..7 hold 4 free: 1, 4, 5, 6 (addresses)
    assert list(fs.addresses(r1)) == [1, 4, 5, 6]
    r2 = fs.reserve(3)              # continues after r1's window
    assert list(fs.addresses(r2)) == [8, 9, 10]
    fs.acquire(fs.addresses(r1)[:2])
    fs.forfeit()
    fs.forfeit()
    r3 = fs.reserve(2)              # a new session starts from the first free block again
    assert list(fs.addresses(r3)) == [5, 6]


def test_level_overlap_and_least_overlap_choice():
    t = forest.Tree(trees.BY_NAME["transfers.id"])

    def info(lo, hi, addr):
        return TableInfo(lo, hi, addr, addr, 16, SNAPSHOT_LATEST, 10, 8, 0)
    for i in range(8):
        t.levels[0].insert(info(100 * i, 100 * i + 50, i + 1))
    t.levels[1].insert(info(0, 120, 20))
    t.levels[1].insert(info(130, 260, 21))
    assert t.levels[1].overlapping(110, 140, 8)[2] == [t.levels[1].tables[0], t.levels[1].tables[1]]
    assert t.levels[1].overlapping(110, 140, 1) is None
    a, r = t.compaction_table(0)
    assert a.key_min == 300 and r[2] == []  # the first table with no overlap: a move
    assert t.compaction_table(1) is None    # level 1 is below its 64 tables


def test_benchmark_load_shape():
    load = benchmark_load.BenchmarkLoad(account_count=100, transfer_count=1000, batch=300)
    ops = list(load.ops())
    assert [o.operation for o in ops] == ["register", "create_accounts"] + ["create_transfers"] * 4
    acc = ops[1].puts
    assert len(acc["accounts.id"]) == 100 and len(acc["accounts.ledger"]) == 100
    assert "accounts.user_data_64" not in acc  # zero fields are not indexed (groove.zig:928-934)
    t = ops[2].puts["transfers.timestamp"]
    w = t.view(np.uint64)
    assert list(w[:, 0][:3]) == [1, 2, 3]                      # ids 1.. (identity permutation)
    assert (w[:, 2] != w[:, 4]).all()                          # debit != credit
    assert ((w[:, 2] >= 1) & (w[:, 2] <= 100)).all()
    assert (w[:, 6] >= 1).all()                                # amount +| 1
    assert (t[:, 112:116].view(np.uint32) == 2).all()          # ledger 2
    ts = w[:, 15]
    assert (np.diff(ts.astype(np.int64)) == 1).all()           # prepare_timestamp - len + i + 1
    assert "transfers.pending_id" not in ops[2].puts and "transfers.timeout" not in ops[2].puts
    assert len(ops[2].puts["accounts.timestamp"]) == 2 * 300   # dr, cr update per transfer
    # balances accumulate: the last put of an account carries the sum of its amounts
    dr = w[:, 2]
    amounts = w[:, 6]
    a0 = dr[0]
    puts = ops[2].puts["accounts.timestamp"].view(np.uint64)
    last = puts[puts[:, 0] == a0][-1]
    cr_sum = sum(int(x) for x in amounts[w[:, 4] == a0])
    assert int(last[4]) == int(amounts[dr == a0].sum()) and int(last[8]) == cr_sum
    # deterministic: the same seed gives the same bytes
    again = list(benchmark_load.BenchmarkLoad(account_count=100, transfer_count=1000, batch=300).ops())
    assert np.array_equal(again[3].puts["transfers.user_data_128"], ops[3].puts["transfers.user_data_128"])


def test_small_benchmark_replay_on_the_oracle(oracle_lib):
    """14 bars of a scaled-down benchmark (64 transfers per op) through the
    Forest schedule: immutable flushes, level-0 merges, moves into level 1;
    every tree's levels stay sorted, disjoint and within their table counts,
    and all values put are found again (newest version per key)."""
    ex = OracleExecutor(oracle_lib)
    f = forest.Forest(ex, block_count=1 << 16, cluster=7)
    load = benchmark_load.BenchmarkLoad(account_count=300, transfer_count=64 * 32 * 14, batch=64)
    f.run(load.ops())
    kinds = {(c.table_a is None, c.move) for _, cs in f.history for _, c in cs}
    assert (True, False) in kinds and (False, True) in kinds  # immutable flushes and moves happened
    for name, t in f.trees.items():
        for level, lv in enumerate(t.levels):
            tabs = lv.visible()
            assert len(tabs) <= forest.table_count_max_for_level(level) + 1
            for x, y in zip(tabs, tabs[1:]):
                assert x.key_max < y.key_min, (name, level)
    # transfers.id: every transfer id flushed to disk is present exactly once
    t = f.trees["transfers.id"]
    spec = t.spec
    vals = []
    for lv in t.levels:
        for info in lv.visible():
            vals.extend(ex.table_segments(info, spec))
    ids = np.concatenate([v.view(np.uint64)[:, 0] for v in vals])
    assert len(ids) == len(np.unique(ids))
    # bars are flushed in order: the ids on disk are a prefix 1..F of the transfers
    assert len(ids) > 0 and np.array_equal(np.sort(ids), np.arange(1, len(ids) + 1, dtype=np.uint64))
    # accounts.timestamp: one (latest) version per account on disk per level range
    acc = f.trees["accounts.timestamp"]
    keys = []
    for lv in acc.levels:
        for info in lv.visible():
            for s in ex.table_segments(info, acc.spec):
                keys.extend(workloads.keys_of(s, acc.spec)[0].tolist())
    assert len(keys) > 0


def test_replay_manifest_log_recovers_the_forest(oracle_lib):
    """The manifest events of a replay (apply_to_manifest + remove_invisible_tables,
    forest.py Tree.apply) through the ManifestLog: after its checkpoint,
    ManifestLog.open's reverse scan and the chronological replay of every
    block both recover exactly the tables in the forest's levels, at their
    levels and snapshots (Forest.verify_tables_recovered, forest.zig:560-650),
    and the log's extents cover every table (verify_table_extents)."""
    from tigerbeetle_amd import manifest
    ex = OracleExecutor(oracle_lib)
    f = forest.Forest(ex, block_count=1 << 16, cluster=7)
    load = benchmark_load.BenchmarkLoad(account_count=300, transfer_count=64 * 32 * 10, batch=64)
    f.run(load.ops())
    if f.pending is not None:   # finish the running half-bar
        op = f.pending[1][0][1].op_min + forest.HALF - 1
        f.compact(op)
    log = f.manifest_log
    assert log.stats["appends"] > 0
    f.checkpoint_manifest()
    blocks = [ex.grid[a] for a in log.log_addresses]
    assert blocks
    opened = manifest.open_log(blocks)
    replayed = manifest.replay_log(blocks)
    want = {}
    for name, t in f.trees.items():
        for level, lv in enumerate(t.levels):
            for info in lv.tables:
                want[info.address] = info.encode(t.spec.tree_id, level, 1, t.spec.key_size)
    assert set(opened) == set(want) == set(log.table_extents)
    for a, e in want.items():   # same table, level, snapshots (the label's event may be insert or update)
        got = opened[a].copy()
        got[126] &= 0x3f
        e = e.copy()
        e[126] &= 0x3f
        assert np.array_equal(got, e), a
    assert {int(e[96:104].view(np.uint64)[0]) for e in replayed.values()} == set(want)
    # events by kind: inserts of outputs, updates of inputs and moves, removes of inputs
    kinds = {}
    for blk in blocks:
        n = int(blk[168:172].view(np.uint32)[0])
        for e in blk[256:256 + 128 * n].reshape(n, 128):
            kinds[int(e[126]) >> 6] = kinds.get(int(e[126]) >> 6, 0) + 1
    assert kinds.get(1, 0) > 0 and kinds.get(2, 0) > 0 and kinds.get(3, 0) > 0


def _levels(f):
    return {name: [[(i.address, i.key_min, i.key_max, i.snapshot_min, i.snapshot_max, i.value_count)
                    for i in lv.tables] for lv in t.levels] for name, t in f.trees.items()}


def test_checkpoint_frees_released_blocks_and_restart_replays_deterministically(oracle_lib):
    """Checkpoints every 2 bars (a short vsr_checkpoint_interval): blocks
    released by compactions and by manifest-log compaction are staged, freed
    at the checkpoint (free_set.zig:383-390, 434-447) and reused by later
    reservations. A crash 1.3 bars after a checkpoint, then a restart from it
    (checkpointed manifest, free set and log; empty memtables) that replays
    the ops after the checkpoint — skipping the compactions the checkpoint
    holds (tree.zig:627-646) — must redo the lost half-bars identically and
    end in the same manifest, free set and log as an uninterrupted run."""
    interval = 2 * forest.BAR
    load = benchmark_load.BenchmarkLoad(account_count=300, transfer_count=64 * 32 * 9, batch=64)
    f1 = forest.Forest(OracleExecutor(oracle_lib), block_count=1 << 16, cluster=7, checkpoint_interval=interval)
    f1.run(load.ops())
    assert [c[:2] for c in f1.checkpoints][:3] == [(63, 95), (127, 159), (191, 223)]
    assert all(freed > 0 for _, _, freed in f1.checkpoints[1:])
    assert f1.free_set.reused > 0            # freed addresses were acquired again

    ex2 = OracleExecutor(oracle_lib)
    f2 = forest.Forest(ex2, block_count=1 << 16, cluster=7, checkpoint_interval=interval)
    crash = 159 + 42
    f2.run(load.ops(), stop=crash)
    before = {op: [c.outputs for _, c in cs] for op, cs in f2.history if op > 159}
    assert before, "half-bars completed after the checkpoint's trigger op before the crash"
    start = f2.restart()
    assert start == 128 and f2.op_compacted_max == 159
    n_hist = len(f2.history)
    f2.run(load.ops(), start=start)
    redone = {op: [c.outputs for _, c in cs] for op, cs in f2.history[n_hist:] if op in before}
    assert redone == before                     # the lost half-bars, byte-identical TableInfos
    assert all(not cs for op, cs in f2.history[n_hist:] if op <= 159)  # skipped: in the checkpoint
    assert [c[:2] for c in f2.checkpoints] == [c[:2] for c in f1.checkpoints]
    assert _levels(f2) == _levels(f1)
    assert np.array_equal(f2.free_set.acquired, f1.free_set.acquired)
    assert list(f2.manifest_log.log_addresses) == list(f1.manifest_log.log_addresses)
    assert f2.manifest_log.table_extents == f1.manifest_log.table_extents
