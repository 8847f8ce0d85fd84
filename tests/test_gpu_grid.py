"""GPU-resident grid and device memtables (row 2).

Two half-bars chained through the grid: batch 1's output tables (left in
HBM) are batch 2's inputs, named only by their TableInfo as Compaction.Context
does; tables "read from storage" are staged with tbc_grid_put_blocks and
validated by the batch that reads them. Every output block and TableInfo is
compared byte for byte with the oracle run on the same values and addresses.
"""

import numpy as np
import pytest

from helpers import disk_image, oracle_tree
from tigerbeetle_amd import Grid, Job, Memtable, abi, trees, workloads
from tigerbeetle_amd.tables import TableInfo

pytestmark = pytest.mark.gpu

BS = 1 << 20
CLUSTER = 0xC1A5


def storage_table(oracle_lib, spec, values, addresses, level=1):
    """A valid on-disk table (data blocks + index block) of sorted unique values,
    built by the oracle as an immutable flush: (block images, TableInfo)."""
    t = oracle_tree(oracle_lib, spec, BS)
    o = oracle_lib.compact(t, [values], [], a_immutable=True, drop_tombstones=False, level_b=level,
                           cluster=CLUSTER, snapshot_min=32, addresses=addresses)
    assert o.status == 0 and len(o.table_infos) == 1
    return o.blocks, TableInfo.decode(o.table_infos[0], spec.key_size)


def table_values(blocks, spec):
    vals = [b[256:int(b[96:100].view(np.uint32)[0])].reshape(-1, spec.value_size) for b in blocks if b[240] == 5]
    return np.concatenate(vals) if vals else np.zeros((0, spec.value_size), np.uint8)


def sorted_unique(spec, n, rng, **kw):
    limbs = workloads.unique_sorted_keys(spec, n, rng, **kw)
    return workloads.values_from_keys(spec, limbs, np.zeros(n, dtype=bool), rng)


def check_job(oracle_lib, grid, spec, r, infos, a_vals, a_immutable, b_tables_vals, drop, level_b, snapshot_min,
              addrs):
    t = oracle_tree(oracle_lib, spec, BS)
    vcm = t.block_value_count_max
    segs_a = [a_vals] if a_immutable else workloads.split_blocks(a_vals, vcm)
    segs_b = [blk for tb in b_tables_vals for blk in workloads.split_blocks(tb, vcm)]
    o = oracle_lib.compact(t, segs_a, segs_b, a_immutable=a_immutable, drop_tombstones=drop, level_b=level_b,
                           cluster=CLUSTER, snapshot_min=snapshot_min, addresses=addrs)
    assert o.status == 0 and r.status == 0
    assert r.block_count == len(o.blocks) and r.value_count == o.value_count
    got = grid.get_blocks(addrs[:r.block_count])
    for g, w in zip(got, o.blocks):
        assert np.array_equal(disk_image(g), disk_image(w))
    assert np.array_equal(infos, o.table_infos)
    return o


def test_two_half_bars_chained_through_the_grid(engine, oracle_lib):
    rng = np.random.default_rng(0x6A1D)
    grid = Grid(engine, 600)
    spec_id = trees.BY_NAME["transfers.id"]
    spec_acc = trees.BY_NAME["accounts.timestamp"]
    try:
        # Storage: two level-0 tables of transfers.id and an accounts table.
        universe = sorted_unique(spec_id, 160_000, rng)
        pick = np.zeros(len(universe), bool)
        pick[rng.choice(len(universe), 90_000, replace=False)] = True
        b_all = universe[~pick]
        b1, b2 = b_all[: len(b_all) // 2], b_all[len(b_all) // 2:]
        blk1, ti1 = storage_table(oracle_lib, spec_id, b1, np.arange(1, 20, dtype=np.uint64), level=0)
        blk2, ti2 = storage_table(oracle_lib, spec_id, b2, np.arange(20, 40, dtype=np.uint64), level=0)
        acc_b = sorted_unique(spec_acc, 30_000, rng)
        blk3, ti3 = storage_table(oracle_lib, spec_acc, acc_b, np.arange(40, 60, dtype=np.uint64), level=2)
        acc_a_keys = [workloads.keys_of(acc_b, spec_acc)[0][rng.choice(30_000, 12_000, replace=False)]]
        acc_a_keys[0].sort()
        acc_a = workloads.values_from_keys(spec_acc, acc_a_keys, rng.random(12_000) < 0.1, rng)
        blk4, ti4 = storage_table(oracle_lib, spec_acc, acc_a, np.arange(60, 80, dtype=np.uint64), level=1)
        for blocks, ti, base in ((blk1, ti1, 1), (blk2, ti2, 20), (blk3, ti3, 40), (blk4, ti4, 60)):
            grid.put_blocks(np.arange(base, base + len(blocks), dtype=np.uint64), np.stack(blocks))

        # The bar's memtable (device ingest in put batches, then the bar-end sort).
        mem_vals = universe[pick]
        shuffled = workloads.shuffle_for_memtable(mem_vals, rng, spec_id)
        mem = Memtable(engine, spec_id)
        for lo in range(0, len(shuffled), 8190):
            mem.put(shuffled[lo:lo + 8190])
        mptr, mcount = mem.values()
        assert mcount == len(shuffled)
        engine.sort_values_batch([(spec_id, mptr, mcount)])

        # Half-bar 1: immutable -> L0 (transfers.id) and L1 -> L2 (accounts, last level for the range).
        a1 = np.arange(100, 100 + 3 * 9, dtype=np.uint64)
        a2 = np.arange(200, 200 + 2 * 65, dtype=np.uint64)
        jobs = [Job(spec_id, [(mptr, mcount)], [], True, False, 0, CLUSTER, 48, a1, None,
                    flags=abi.COMPACTION_GRID, grid=grid, tables_b=[ti1.ref(), ti2.ref()]),
                Job(spec_acc, [], [], False, True, 2, CLUSTER, 48, a2, None, flags=abi.COMPACTION_GRID, grid=grid,
                    tables_a=[ti4.ref()], tables_b=[ti3.ref()])]
        b = engine.submit(jobs)
        b.wait()
        (r1, inf1), (r2, inf2) = b.result(0), b.result(1)
        b.release()
        o1 = check_job(oracle_lib, grid, spec_id, r1, inf1, mem_vals, True, [b1, b2], False, 0, 48, a1)
        check_job(oracle_lib, grid, spec_acc, r2, inf2, acc_a, False, [acc_b], True, 2, 48, a2)

        # Half-bar 2: the first output table of job 1 is disk A of an L0 -> L1
        # compaction against a new storage table (inputs read from the grid only).
        out_t0 = TableInfo.decode(inf1[0], spec_id.key_size)
        a_vals = table_values(o1.blocks[:10], spec_id)[: out_t0.value_count]
        assert len(a_vals) == out_t0.value_count
        lo_key, hi_key = out_t0.key_min, out_t0.key_max
        more = sorted_unique(spec_id, 40_000, rng)
        mk = workloads.keys_of(more, spec_id)
        mint = mk[0].astype(object) | (mk[1].astype(object) << 64)
        fresh = more[(mint > lo_key) & (mint < hi_key)]
        in_a = set(map(bytes, a_vals[:, :16]))
        fresh = fresh[[bytes(v[:16]) not in in_a for v in fresh]]
        blk5, ti5 = storage_table(oracle_lib, spec_id, fresh, np.arange(300, 320, dtype=np.uint64), level=1)
        grid.put_blocks(np.arange(300, 300 + len(blk5), dtype=np.uint64), np.stack(blk5))
        a3 = np.arange(400, 400 + 2 * 9, dtype=np.uint64)
        b = engine.submit([Job(spec_id, [], [], False, False, 1, CLUSTER, 64, a3, None, flags=abi.COMPACTION_GRID,
                               grid=grid, tables_a=[out_t0.ref()], tables_b=[ti5.ref()])])
        b.wait()
        r3, inf3 = b.result(0)
        b.release()
        check_job(oracle_lib, grid, spec_id, r3, inf3, a_vals, False, [fresh], False, 1, 64, a3)
        mem.close()
    finally:
        grid.close()


def test_grid_batches_in_flight_together(engine, oracle_lib):
    """Three grid batches submitted back to back with a put_blocks between
    them and no wait: batch 2 reads batch 1's first output table (its fronts
    find the data blocks through the index block batch 1's front laid out
    early; its input checks wait for batch 1's tail), batch 3 reads a storage
    table batch 1 also reads. Expected outputs come from the oracle before
    anything is submitted (the output TableInfo batch 2 names is the
    oracle's)."""
    rng = np.random.default_rng(0x3B47)
    grid = Grid(engine, 700)
    spec_id = trees.BY_NAME["transfers.id"]
    spec_acc = trees.BY_NAME["accounts.timestamp"]
    mem = None
    try:
        universe = sorted_unique(spec_id, 160_000, rng)
        pick = np.zeros(len(universe), bool)
        pick[rng.choice(len(universe), 90_000, replace=False)] = True
        b_all = universe[~pick]
        blk1, ti1 = storage_table(oracle_lib, spec_id, b_all, np.arange(1, 40, dtype=np.uint64), level=0)
        acc_b = sorted_unique(spec_acc, 30_000, rng)
        blk3, ti3 = storage_table(oracle_lib, spec_acc, acc_b, np.arange(40, 60, dtype=np.uint64), level=2)
        acc_keys = workloads.keys_of(acc_b, spec_acc)[0]
        acc_a = workloads.values_from_keys(spec_acc, [np.sort(acc_keys[rng.choice(30_000, 12_000, replace=False)])],
                                           rng.random(12_000) < 0.1, rng)
        blk4, ti4 = storage_table(oracle_lib, spec_acc, acc_a, np.arange(60, 80, dtype=np.uint64), level=1)
        acc_c = workloads.values_from_keys(spec_acc, [np.sort(acc_keys[rng.choice(30_000, 9_000, replace=False)])],
                                           rng.random(9_000) < 0.2, rng)
        blk6, ti6 = storage_table(oracle_lib, spec_acc, acc_c, np.arange(80, 100, dtype=np.uint64), level=1)
        for blocks, ti, base in ((blk1, ti1, 1), (blk3, ti3, 40), (blk4, ti4, 60), (blk6, ti6, 80)):
            grid.put_blocks(np.arange(base, base + len(blocks), dtype=np.uint64), np.stack(blocks))

        mem_vals = universe[pick]
        mem = Memtable(engine, spec_id)
        shuffled = workloads.shuffle_for_memtable(mem_vals, rng, spec_id)
        for lo in range(0, len(shuffled), 8190):
            mem.put(shuffled[lo:lo + 8190])
        mptr, mcount = mem.values()
        engine.sort_values_batch([(spec_id, mptr, mcount)])

        # The oracle first: batch 1's flush decides batch 2's input table.
        a1 = np.arange(100, 100 + 3 * 9, dtype=np.uint64)
        a2 = np.arange(200, 200 + 2 * 65, dtype=np.uint64)
        a3 = np.arange(400, 400 + 2 * 9, dtype=np.uint64)
        a4 = np.arange(500, 500 + 2 * 65, dtype=np.uint64)
        t = oracle_tree(oracle_lib, spec_id, BS)
        o1 = oracle_lib.compact(t, [mem_vals], workloads.split_blocks(b_all, t.block_value_count_max),
                                a_immutable=True, drop_tombstones=False, level_b=0, cluster=CLUSTER,
                                snapshot_min=48, addresses=a1)
        out_t0 = TableInfo.decode(o1.table_infos[0], spec_id.key_size)
        a_vals = table_values(o1.blocks[:10], spec_id)[: out_t0.value_count]
        lo_key, hi_key = out_t0.key_min, out_t0.key_max
        more = sorted_unique(spec_id, 40_000, rng)
        mk = workloads.keys_of(more, spec_id)
        mint = mk[0].astype(object) | (mk[1].astype(object) << 64)
        fresh = more[(mint > lo_key) & (mint < hi_key)]
        in_a = set(map(bytes, a_vals[:, :16]))
        fresh = fresh[[bytes(v[:16]) not in in_a for v in fresh]]
        blk5, ti5 = storage_table(oracle_lib, spec_id, fresh, np.arange(300, 320, dtype=np.uint64), level=1)

        def gjob(spec, level, snap, addrs, drop=False, **kw):
            return Job(spec, kw.pop("segs_a", []), [], kw.pop("imm", False), drop, level, CLUSTER, snap, addrs, None,
                       flags=abi.COMPACTION_GRID, grid=grid, **kw)

        h1 = engine.submit([gjob(spec_id, 0, 48, a1, segs_a=[(mptr, mcount)], imm=True, tables_b=[ti1.ref()]),
                            gjob(spec_acc, 2, 48, a2, drop=True, tables_a=[ti4.ref()], tables_b=[ti3.ref()])])
        grid.put_blocks(np.arange(300, 300 + len(blk5), dtype=np.uint64), np.stack(blk5))
        h2 = engine.submit([gjob(spec_id, 1, 64, a3, tables_a=[out_t0.ref()], tables_b=[ti5.ref()])])
        h3 = engine.submit([gjob(spec_acc, 2, 48, a4, drop=True, tables_a=[ti6.ref()], tables_b=[ti3.ref()])])
        for h in (h3, h2, h1):
            h.wait()
        res = [h1.result(0), h1.result(1), h2.result(0), h3.result(0)]
        for h in (h1, h2, h3):
            h.release()
        check_job(oracle_lib, grid, spec_id, *res[0], mem_vals, True, [b_all], False, 0, 48, a1)
        check_job(oracle_lib, grid, spec_acc, *res[1], acc_a, False, [acc_b], True, 2, 48, a2)
        check_job(oracle_lib, grid, spec_id, *res[2], a_vals, False, [fresh], False, 1, 64, a3)
        check_job(oracle_lib, grid, spec_acc, *res[3], acc_c, False, [acc_b], True, 2, 48, a4)
        # Batch 2 found its input table only through the grid: it was trusted
        # (batch 1's output) or validated, and nothing failed.
        assert all(r.status == 0 for r, _ in res)
    finally:
        if mem is not None:
            mem.close()
        grid.close()


def test_grid_rejects_corrupt_and_unexpected_blocks(engine, oracle_lib):
    """read_block_validate on blocks from storage (a flipped body byte), and
    read_block_from_cache's checksum comparison on trusted blocks (a table
    reference with the wrong checksum): TBC_ERR_BLOCK_INVALID for that job
    only; the others in the batch complete."""
    rng = np.random.default_rng(0xBAD)
    grid = Grid(engine, 200)
    spec = trees.BY_NAME["transfers.id"]
    try:
        vals = sorted_unique(spec, 50_000, rng)
        blocks, ti = storage_table(oracle_lib, spec, vals, np.arange(1, 10, dtype=np.uint64))
        bad = np.stack(blocks).copy()
        bad[1, 256 + 999] ^= 0x40  # a data block body byte
        grid.put_blocks(np.arange(1, 1 + len(blocks), dtype=np.uint64), bad)
        good_vals = sorted_unique(spec, 30_000, rng)
        gblocks, gti = storage_table(oracle_lib, spec, good_vals, np.arange(20, 30, dtype=np.uint64))
        grid.put_blocks(np.arange(20, 20 + len(gblocks), dtype=np.uint64), np.stack(gblocks))

        def job(tref, base):
            return Job(spec, [], [], False, False, 2, CLUSTER, 48, np.arange(base, base + 9, dtype=np.uint64), None,
                       flags=abi.COMPACTION_GRID, grid=grid, tables_a=[tref])

        b = engine.submit([job(ti.ref(), 50), job(gti.ref(), 70)])
        assert b.poll() in (abi.TBC_PENDING, abi.TBC_ERR_BLOCK_INVALID)
        with pytest.raises(abi.TbcError):
            b.wait()
        r0, r1 = b.result(0)[0], b.result(1)[0]
        assert r0.status == abi.TBC_ERR_BLOCK_INVALID and r1.status == 0
        b.release()
        # The good table is now trusted; naming it with a wrong checksum is a miss.
        wrong = (gti.address, gti.checksum ^ 1, gti.value_count)
        b = engine.submit([job(wrong, 90)])
        with pytest.raises(abi.TbcError):
            b.wait()
        assert b.result(0)[0].status == abi.TBC_ERR_BLOCK_INVALID
        b.release()
        # Re-staging the intact table from storage makes it readable again.
        grid.put_blocks(np.arange(1, 1 + len(blocks), dtype=np.uint64), np.stack(blocks))
        b = engine.submit([job(ti.ref(), 110)])
        b.wait()
        assert b.result(0)[0].status == 0
        b.release()
    finally:
        grid.close()


def test_memtable_put_capacity_and_reset(engine):
    spec = trees.with_table_size(trees.BY_NAME["transfers.code"], 1000)
    rng = np.random.default_rng(5)
    vals = workloads.values_from_keys(spec, workloads.random_keys(spec, 1000, rng), np.zeros(1000, bool), rng)
    m = Memtable(engine, spec)
    try:
        m.put(vals[:600])
        m.put(vals[600:])
        with pytest.raises(abi.TbcError) as e:
            m.put(vals[:1])
        assert e.value.status == abi.TBC_ERR_CAPACITY
        ptr, n = m.values()
        assert n == 1000
        got = np.empty(vals.nbytes, np.uint8)
        abi.check(abi.lib().tbc_copy_to_host(engine.handle, got.ctypes.data, ptr, vals.nbytes), "copy")
        assert np.array_equal(got.reshape(vals.shape), vals)
        m.reset()
        assert m.values()[1] == 0
    finally:
        m.close()


def test_grid_unique_keys_held_and_broken(engine, oracle_lib):
    """Grid batches with TBC_COMPACTION_UNIQUE_KEYS jobs: a grid batch does
    not speculate (every job through the mask merge; round 4's and round 6's
    tile-by-tile grid speculation measured slower on config 1),
    so the flag changes nothing: held, repeating and plain jobs alike give
    the oracle's blocks and TableInfos, and tbc_batch_speculation reports
    NONE."""
    rng = np.random.default_rng(0x0A1B)
    grid = Grid(engine, 700)
    spec_id = trees.BY_NAME["transfers.id"]
    spec_ts = trees.BY_NAME["transfers.timestamp"]
    spec_acc = trees.BY_NAME["accounts.timestamp"]
    try:
        uni = sorted_unique(spec_id, 200_000, rng)
        part = rng.integers(0, 3, size=len(uni))
        b_vals, a_vals, c_vals = uni[part == 0], uni[part == 1], uni[part == 2]
        blk_b, ti_b = storage_table(oracle_lib, spec_id, b_vals, np.arange(1, 20, dtype=np.uint64), level=1)
        blk_a, ti_a = storage_table(oracle_lib, spec_id, a_vals, np.arange(20, 40, dtype=np.uint64), level=0)
        # broken: C's table repeats 50 keys of B's
        c_rep = np.concatenate([c_vals, b_vals[rng.choice(len(b_vals), 50, replace=False)]])
        c_rep = c_rep[np.lexsort(workloads.keys_of(c_rep, spec_id))]  # most significant limb last
        blk_c, ti_c = storage_table(oracle_lib, spec_id, c_rep, np.arange(40, 60, dtype=np.uint64), level=0)
        ts_b = sorted_unique(spec_ts, 60_000, rng)
        blk_t, ti_t = storage_table(oracle_lib, spec_ts, ts_b, np.arange(60, 80, dtype=np.uint64), level=1)
        ts_a = sorted_unique(spec_ts, 30_000, rng)
        mem_ts = engine.upload(ts_a)
        acc_b = sorted_unique(spec_acc, 20_000, rng)
        blk_acc, ti_acc = storage_table(oracle_lib, spec_acc, acc_b, np.arange(80, 100, dtype=np.uint64), level=2)
        acc_keys = [np.sort(workloads.keys_of(acc_b, spec_acc)[0][rng.choice(20_000, 5_000, replace=False)])]
        acc_a = workloads.values_from_keys(spec_acc, acc_keys, np.zeros(5_000, bool), rng)
        mem_acc = engine.upload(acc_a)
        for blocks, base in ((blk_b, 1), (blk_a, 20), (blk_c, 40), (blk_t, 60), (blk_acc, 80)):
            grid.put_blocks(np.arange(base, base + len(blocks), dtype=np.uint64), np.stack(blocks))
        U, G = abi.COMPACTION_UNIQUE_KEYS, abi.COMPACTION_GRID
        adr = [np.arange(b, b + n, dtype=np.uint64) for b, n in ((200, 27), (300, 27), (400, 18), (500, 130))]
        jobs = [Job(spec_id, [], [], False, False, 1, CLUSTER, 48, adr[0], None, flags=G | U, grid=grid,
                    tables_a=[ti_a.ref()], tables_b=[ti_b.ref()]),                      # held
                Job(spec_id, [], [], False, False, 1, CLUSTER, 48, adr[1], None, flags=G | U, grid=grid,
                    tables_a=[ti_c.ref()], tables_b=[ti_b.ref()]),                      # broken
                Job(spec_ts, [(mem_ts.ptr, len(ts_a))], [], True, False, 1, CLUSTER, 48, adr[2], None,
                    flags=G | U, grid=grid, tables_b=[ti_t.ref()]),                     # held, immutable A
                Job(spec_acc, [(mem_acc.ptr, len(acc_a))], [], True, True, 2, CLUSTER, 48, adr[3], None,
                    flags=G, grid=grid, tables_b=[ti_acc.ref()])]                       # mask merge
        b = engine.submit(jobs)
        b.wait()
        res = [b.result(i) for i in range(4)]
        spec_out = [b.speculation(i) for i in range(4)]
        b.release()
        assert spec_out == [abi.SPECULATION_NONE] * 4
        check_job(oracle_lib, grid, spec_id, *res[0], a_vals, False, [b_vals], False, 1, 48, adr[0])
        check_job(oracle_lib, grid, spec_id, *res[1], c_rep, False, [b_vals], False, 1, 48, adr[1])
        check_job(oracle_lib, grid, spec_ts, *res[2], ts_a, True, [ts_b], False, 1, 48, adr[2])
        check_job(oracle_lib, grid, spec_acc, *res[3], acc_a, True, [acc_b], True, 2, 48, adr[3])
    finally:
        grid.close()
