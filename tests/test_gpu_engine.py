"""Engine-level behaviour that the per-kernel parity tests do not reach.

- The static arenas (engine.hip Arena): batches and k-way merges open a
  region at submit and close it at release. With one batch held live (the
  adapter always has something in flight), many submit/release cycles of
  k-way merges and batches must not grow the arenas' tops, and regions
  released out of order are reclaimed once the ones above them are.
- Pipelined grid batches (engine.hip submit_impl, grid mode): several
  half-bars' batches in flight at once, submitted back to back without
  waiting, with a storage stage (tbc_grid_put_blocks) between two submits,
  later batches reading storage tables that earlier ones also read (the
  first reader validates them in full, later readers must see them
  trusted), and one corrupt storage table. Every job's blocks and TableInfos
  are compared with the oracle; the corrupt table's job alone fails.
- Failed grid jobs leave their outputs unverified (k_grid_mark runs after
  the input checks, and only for clean jobs): a later reader of such an
  output revalidates it in full, while a clean job's outputs are trusted
  like the reference's grid cache hits (grid.zig:802-841).
"""
import numpy as np
import pytest

from test_gpu_grid import BS, CLUSTER, check_job, sorted_unique, storage_table
from tigerbeetle_amd import Grid, Job, abi, trees, workloads

pytestmark = pytest.mark.gpu


def _small_job(engine, spec, rng, n=20_000):
    vals = sorted_unique(spec, n, rng)
    buf = engine.upload(vals)
    out = engine.alloc(4 * BS)
    return buf, out, Job(spec, [(buf.ptr, n)], [], True, False, 1, CLUSTER, 48,
                         np.arange(1, 5, dtype=np.uint64), out)


def test_arena_bounded_with_a_batch_in_flight(engine):
    spec = trees.BY_NAME["transfers.id"]
    rng = np.random.default_rng(0xA7E)
    base = engine.arena_usage()
    keep0 = _small_job(engine, spec, rng)
    held = engine.submit([keep0[2]])          # stays live for the whole loop
    after_held = engine.arena_usage()
    assert after_held[2] == base[2] + 2       # one device + one pinned region
    streams = [sorted_unique(spec, 5_000, rng) for _ in range(4)]
    bufs = [engine.upload(s) for s in streams]
    segs = [(b.ptr, len(s)) for b, s in zip(bufs, streams)]
    kout = engine.alloc(20_000 * 32)
    keep1 = _small_job(engine, spec, rng)
    peak = (0, 0)
    for _ in range(40):
        k = engine.kway_merge_submit(spec, segs, kout)
        b = engine.submit([keep1[2]])
        peak = max(peak, engine.arena_usage()[:2])
        b.wait()
        k.wait()
        assert k.count() == 20_000
        k.release()                            # released below the batch: reclaimed with it
        b.release()
        assert engine.arena_usage() == after_held
    assert peak[0] < after_held[0] + (1 << 20) and peak[1] < after_held[1] + (1 << 20)
    # Out of order: the older region is reclaimed as soon as it closes.
    b1, b2 = engine.submit([keep1[2]]), engine.submit([keep1[2]])
    b1.wait()
    b2.wait()
    top2 = engine.arena_usage()
    b1.release()
    mid = engine.arena_usage()
    assert mid[0] < top2[0] and mid[1] < top2[1] and mid[2] == top2[2] - 2
    b2.release()
    assert engine.arena_usage() == after_held
    held.wait()
    held.release()
    assert engine.arena_usage() == base


def test_arena_reclaims_a_pipelined_stream_of_batches(engine):
    """A caller that always keeps batches in flight and releases the oldest
    first (a replica's steady state): the arena's use stays that of the
    batches in flight over many times its size in total (round 4's stack
    reclaimed nothing until every newer region closed, and ran out)."""
    spec = trees.BY_NAME["transfers.id"]
    rng = np.random.default_rng(0xA7F)
    base = engine.arena_usage()
    jobs = [_small_job(engine, spec, rng) for _ in range(3)]
    b = engine.submit([jobs[0][2]])
    one = [u - v for u, v in zip(engine.arena_usage()[:2], base[:2])]  # one batch's device and pinned bytes
    b.wait()
    b.release()
    pending, peak = [], (0, 0)
    for i in range(600):
        pending.append(engine.submit([jobs[i % 3][2]]))
        peak = max(peak, engine.arena_usage()[:2])
        if len(pending) == 3:
            b = pending.pop(0)
            b.wait()
            assert b.result(0)[0].status == 0
            b.release()
    for b in pending:
        b.wait()
        b.release()
    assert engine.arena_usage() == base
    assert peak[0] <= base[0] + 3 * one[0] and peak[1] <= base[1] + 3 * one[1]


def test_pipelined_grid_batches_in_flight(engine, oracle_lib):
    rng = np.random.default_rng(0x919E)
    grid = Grid(engine, 900)
    sid = trees.BY_NAME["transfers.id"]
    sacc = trees.BY_NAME["accounts.timestamp"]
    try:
        # Storage: S1, S2 (transfers.id, level 1), S3 (accounts, level 2); S4 corrupt.
        uni = sorted_unique(sid, 240_000, rng)
        part = rng.integers(0, 4, size=len(uni))
        s1v, s2v, m1v, m2v = (uni[part == p] for p in range(4))
        blk1, ti1 = storage_table(oracle_lib, sid, s1v, np.arange(1, 12, dtype=np.uint64))
        blk2, ti2 = storage_table(oracle_lib, sid, s2v, np.arange(20, 31, dtype=np.uint64))
        s3v = sorted_unique(sacc, 40_000, rng)
        blk3, ti3 = storage_table(oracle_lib, sacc, s3v, np.arange(40, 60, dtype=np.uint64), level=2)
        s4v = sorted_unique(sid, 30_000, rng)
        blk4, ti4 = storage_table(oracle_lib, sid, s4v, np.arange(60, 70, dtype=np.uint64))
        bad4 = np.stack(blk4).copy()
        bad4[0, 256 + 77] ^= 1
        grid.put_blocks(np.arange(1, 1 + len(blk1), dtype=np.uint64), np.stack(blk1))
        grid.put_blocks(np.arange(20, 20 + len(blk2), dtype=np.uint64), np.stack(blk2))
        grid.put_blocks(np.arange(60, 60 + len(bad4), dtype=np.uint64), bad4)
        m1 = engine.upload(m1v)
        m2 = engine.upload(m2v)
        acc_keys = [np.sort(workloads.keys_of(s3v, sacc)[0][rng.choice(len(s3v), 9_000, replace=False)])]
        acc_a = workloads.values_from_keys(sacc, acc_keys, rng.random(9_000) < 0.05, rng)
        acc_buf = engine.upload(acc_a)

        def grid_job(spec, segs_a, tables_a, tables_b, level_b, drop, base, count):
            return Job(spec, segs_a, [], bool(segs_a), drop, level_b, CLUSTER, 64,
                       np.arange(base, base + count, dtype=np.uint64), None, flags=abi.COMPACTION_GRID, grid=grid,
                       tables_a=tables_a, tables_b=tables_b)

        # Batch 1: immutable M1 into S1 (validates S1), and immutable M2 into S2.
        j1 = [grid_job(sid, [(m1.ptr, len(m1v))], [], [ti1.ref()], 1, False, 100, 3 * 9),
              grid_job(sid, [(m2.ptr, len(m2v))], [], [ti2.ref()], 1, False, 140, 3 * 9)]
        b1 = engine.submit(j1)
        # A storage read between submits (joins the running tails on the engine stream).
        grid.put_blocks(np.arange(40, 40 + len(blk3), dtype=np.uint64), np.stack(blk3))
        # Batch 2: S2 again (as disk A, into nothing below), and the accounts
        # immutable into S3 at the last level.
        j2 = [grid_job(sid, [], [ti2.ref()], [], 2, False, 200, 2 * 9),
              grid_job(sacc, [(acc_buf.ptr, len(acc_a))], [], [ti3.ref()], 3, True, 240, 3 * 65)]
        b2 = engine.submit(j2)
        # Batch 3: S1 again (trusted by now), and the corrupt S4.
        j3 = [grid_job(sid, [], [ti1.ref()], [], 2, False, 500, 2 * 9),
              grid_job(sid, [], [ti4.ref()], [], 2, False, 540, 2 * 9)]
        b3 = engine.submit(j3)
        for b in (b1, b2):
            b.wait()
        with pytest.raises(abi.TbcError):
            b3.wait()
        res = [b.result(i) for b in (b1, b2, b3) for i in range(2)]
        for b in (b1, b2, b3):
            b.release()
        check_job(oracle_lib, grid, sid, *res[0], m1v, True, [s1v], False, 1, 64, j1[0].addresses)
        check_job(oracle_lib, grid, sid, *res[1], m2v, True, [s2v], False, 1, 64, j1[1].addresses)
        check_job(oracle_lib, grid, sid, *res[2], s2v, False, [], False, 2, 64, j2[0].addresses)
        check_job(oracle_lib, grid, sacc, *res[3], acc_a, True, [s3v], True, 3, 64, j2[1].addresses)
        check_job(oracle_lib, grid, sid, *res[4], s1v, False, [], False, 2, 64, j3[0].addresses)
        assert res[5][0].status == abi.TBC_ERR_BLOCK_INVALID
    finally:
        grid.close()


def test_failed_job_outputs_stay_unverified(engine, oracle_lib):
    rng = np.random.default_rng(0xF00D)
    grid = Grid(engine, 300)
    spec = trees.BY_NAME["transfers.id"]
    try:
        bad_vals = sorted_unique(spec, 50_000, rng)
        blocks, ti = storage_table(oracle_lib, spec, bad_vals, np.arange(1, 10, dtype=np.uint64))
        bad = np.stack(blocks).copy()
        bad[1, 256 + 999] ^= 0x40
        grid.put_blocks(np.arange(1, 1 + len(bad), dtype=np.uint64), bad)
        good_vals = sorted_unique(spec, 30_000, rng)
        gblocks, gti = storage_table(oracle_lib, spec, good_vals, np.arange(20, 30, dtype=np.uint64))
        grid.put_blocks(np.arange(20, 20 + len(gblocks), dtype=np.uint64), np.stack(gblocks))

        def job(tref, base, level=2):
            return Job(spec, [], [], False, False, level, CLUSTER, 48, np.arange(base, base + 9, dtype=np.uint64),
                       None, flags=abi.COMPACTION_GRID, grid=grid, tables_a=[tref])

        b = engine.submit([job(ti.ref(), 50), job(gti.ref(), 70)])
        with pytest.raises(abi.TbcError):
            b.wait()
        (r_bad, inf_bad), (r_good, inf_good) = b.result(0), b.result(1)
        b.release()
        assert r_bad.status == abi.TBC_ERR_BLOCK_INVALID and r_good.status == 0
        from tigerbeetle_amd.tables import TableInfo
        t_bad = TableInfo.decode(inf_bad[0], spec.key_size)
        t_good = TableInfo.decode(inf_good[0], spec.key_size)
        # Flip a body byte of the first data block of each output table in HBM
        # (slot 0 of each job's reservation: addresses 50 and 70).
        for addr in (50, 70):
            ptr = grid.pointer(addr)
            abi.check(abi.lib().tbc_memset_device(engine.handle, ptr + 256 + 5, 0x5A, 1), "memset")
        # The failed job's output is unverified: its reader validates it in
        # full and finds the body checksum broken.
        b = engine.submit([job(t_bad.ref(), 100, 3)])
        with pytest.raises(abi.TbcError):
            b.wait()
        assert b.result(0)[0].status == abi.TBC_ERR_BLOCK_INVALID
        b.release()
        # The clean job's output is trusted (a cache hit: header checksum,
        # address and header fields only), as the reference's grid cache is.
        b = engine.submit([job(t_good.ref(), 130, 3)])
        b.wait()
        assert b.result(0)[0].status == 0
        b.release()
    finally:
        grid.close()


@pytest.mark.gpu
def test_copy_device_batch(engine):
    """tbc_copy_device_batch: aligned copies in one launch (chunked at 64 KiB),
    unaligned ones as copies of their own, sizes from 16 bytes to several
    chunks; the bytes around each destination stay untouched."""
    rng = np.random.default_rng(41)
    sizes = [16, 48, 65536, 65536 + 16, 3 * 65536 + 4096, 1 << 20, 7, 1000]
    src = engine.upload(rng.integers(0, 256, sum(sizes) + 64 * len(sizes), dtype=np.uint8))
    dst = engine.alloc(sum(sizes) + 64 * len(sizes))
    dst.zero()
    copies, so, do = [], 0, 0
    for n in sizes:
        shift = 1 if n % 16 else 0  # the unaligned ones: an odd offset too
        copies.append((dst.ptr + do + shift, src.ptr + so + shift, n))
        so += n + 64
        do += n + 64
    engine.copy_device_batch(copies)
    engine.synchronize()
    s, d = src.download(), dst.download()
    want = np.zeros_like(d)
    off = 0
    for n in sizes:
        shift = 1 if n % 16 else 0
        want[off + shift:off + shift + n] = s[off + shift:off + shift + n]
        off += n + 64
    assert np.array_equal(d, want)


def test_copy_batch_descriptors_survive_kway_scratch_growth():
    """growing the k-way scratch must leave the copy
    batch's descriptor buffer alone. On a fresh engine: a copy batch (its
    descriptor buffer allocated), a k-way merge large enough to grow the
    k-way scratch, another copy batch with data checks, then deinit."""
    from tigerbeetle_amd import Engine
    eng = Engine(device=0, block_size=1 << 20)
    try:
        rng = np.random.default_rng(0xC0DE)
        spec = trees.BY_NAME["transfers.id"]

        def copy_round(seed):
            data = np.random.default_rng(seed).integers(0, 256, 3 << 20, dtype=np.uint8)
            src = eng.upload(data)
            dst = eng.alloc(len(data))
            dst.zero()
            eng.copy_device_batch([(dst.ptr + o, src.ptr + o, 1 << 20) for o in (0, 1 << 20, 2 << 20)])
            eng.synchronize()
            assert np.array_equal(dst.download(), data)

        copy_round(1)
        limbs = workloads.unique_sorted_keys(spec, 400_000, rng)
        streams, idxs = [], []
        for _ in range(4):
            idx = np.sort(rng.choice(400_000, 100_000, replace=False))
            idxs.append(idx)
            streams.append(workloads.values_from_keys(spec, [l[idx] for l in limbs], np.zeros(len(idx), bool), rng))
        bufs = [eng.upload(s) for s in streams]
        out = eng.alloc(400_000 * 32)
        n = eng.kway_merge(spec, [(b.ptr, len(s)) for b, s in zip(bufs, streams)], out)
        assert n == len(np.unique(np.concatenate(idxs)))  # one value per distinct key
        copy_round(2)
        copy_round(3)
    finally:
        eng.close()


def test_grid_block_transfers_staged_and_registered(engine):
    """tbc_grid_put_blocks / tbc_grid_get_blocks (round 4: the D2H ring keeps
    every slot in flight; registered host ranges go by direct DMA): 20 blocks
    (more than the 8 staging slots) round-trip byte for byte through pageable
    memory, through host-registered arrays, and mixed; the verified bytes of
    staged blocks are cleared by one launch (a later trusted check fails)."""
    bs = engine.block_size
    grid = Grid(engine, 64)
    try:
        rng = np.random.default_rng(0x9C1E)
        n = 20
        addrs = rng.permutation(np.arange(1, 65, dtype=np.uint64))[:n]
        imgs = rng.integers(0, 256, size=(n, bs), dtype=np.uint8)
        grid.put_blocks(addrs, imgs)
        assert np.array_equal(grid.get_blocks(addrs), imgs)
        reg_in = rng.integers(0, 256, size=(n, bs), dtype=np.uint8)
        reg_out = np.zeros_like(reg_in)
        engine.host_register(reg_in)
        engine.host_register(reg_out)
        try:
            grid.put_blocks(addrs, reg_in)
            got = grid.get_blocks(addrs, out=reg_out)
            assert np.shares_memory(got, reg_out) and np.array_equal(reg_out, reg_in)
            with pytest.raises(abi.TbcError):  # overlapping registration refused
                engine.host_register(reg_in[1:3])
        finally:
            engine.host_unregister(reg_in)
            engine.host_unregister(reg_out)
        assert np.array_equal(grid.get_blocks(addrs[::-1]), reg_in[::-1])
    finally:
        grid.close()
