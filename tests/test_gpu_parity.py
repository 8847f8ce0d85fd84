"""GPU parity: libtbc.so (HIP, gfx950) against the CPU oracle, bit-exact.

Checksums are compared with the reference KATs (src/vsr/checksum.zig:94-195)
and the oracle; compactions compare every output block's on-disk image
(block[0..sector_ceil(size)], grid.zig:686 / storage_checker.zig:305-310)
and every TableInfo (schema.zig:489-509) with the oracle's restatement of
compaction.zig/table.zig.
"""
import numpy as np
import pytest

import zig_prng
from helpers import disk_image, gpu_run, run_oracle
from tigerbeetle_amd import abi, trees, workloads

pytestmark = pytest.mark.gpu


def bswap128(x):
    return int.from_bytes(x.to_bytes(16, "big"), "little")


def test_checksum_test_vectors(engine):
    got = engine.checksum([bytes(16), b""])
    assert got[0] == bswap128(0xF72AD48DD05DD1656133101CD4BE3A26)
    assert got[1] == 0x49F174618255402DE6E7E3C40D60CC83


def test_checksum_stability(engine):
    msgs = zig_prng.stability_messages()
    cases = engine.checksum(msgs)
    blob = b"".join(c.to_bytes(16, "little") for c in cases)
    assert engine.checksum([blob])[0] == zig_prng.STABILITY_HASH


def test_checksum_random_lengths(engine, oracle_lib):
    rng = np.random.default_rng(5)
    lens = [0, 1, 15, 16, 17, 31, 32, 33, 240, 255, 256, 257, 1000, 4096, 65536 + 3, 1048320]
    lens += [int(x) for x in rng.integers(1, 300_000, size=8)]
    msgs = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    got = engine.checksum(msgs)
    for m, g in zip(msgs, got):
        assert g == oracle_lib.checksum(m), len(m)


def _compare(oracle_lib, engine, cases, block_size, level_b=1):
    """Run all cases as ONE batch on the GPU; compare each with the oracle."""
    rng = np.random.default_rng(99)
    inputs, addrs = [], []
    for (spec, kw) in cases:
        ji = workloads.make_job_inputs(spec, rng, **kw)
        n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
        addrs.append(workloads.addresses_for(workloads.worst_case_blocks(spec, n, block_size) + 3, rng,
                                             int(rng.integers(1, 1000)), 0.1))
        inputs.append(ji)
    results, _ = gpu_run(engine, inputs, block_size, addrs, level_b=level_b)
    for ji, a, (r, infos, blocks) in zip(inputs, addrs, results):
        o = run_oracle(oracle_lib, ji, block_size, a, level_b=level_b)
        assert o.status == 0
        assert r.status == 0
        assert (r.value_count, r.data_block_count, r.table_count, r.block_count) == \
               (o.value_count, o.data_block_count, len(o.table_infos), len(o.blocks)), ji.tree.name
        for i, (g, w) in enumerate(zip(blocks, o.blocks)):
            gi, wi = disk_image(g), disk_image(w)
            if not np.array_equal(gi, wi):
                diff = np.nonzero(gi[: len(wi)] != wi[: len(gi)])[0]
                raise AssertionError(f"{ji.tree.name}: block {i} differs at bytes {diff[:16]} "
                                     f"(type {w[240]}, size {len(wi)})")
        assert np.array_equal(infos, o.table_infos)


SMALL = [
    ("transfers.id", dict(n_a=2000, b_table_sizes=[700, 900, 300], a_immutable=False, overlap=0.3)),
    ("transfers.id", dict(n_a=2500, b_table_sizes=[1200], a_immutable=True, dup_frac=0.2, tomb_frac=0.1,
                          drop_tombstones=True, overlap=0.5)),
    ("transfers.timestamp", dict(n_a=900, b_table_sizes=[100, 150, 90], a_immutable=True, dup_frac=0.3,
                                 tomb_frac=0.2, overlap=0.4)),
    ("transfers.timestamp", dict(n_a=700, b_table_sizes=[], a_immutable=False, tomb_frac=0.3,
                                 drop_tombstones=True)),
    ("transfers.debit_account_id", dict(n_a=3000, b_table_sizes=[800, 900], a_immutable=True, dup_frac=0.4,
                                        drop_tombstones=True, overlap=0.3)),
    ("accounts.ledger", dict(n_a=2600, b_table_sizes=[1500], a_immutable=True, dup_frac=0.3, overlap=0.5)),
    ("posted.timestamp", dict(n_a=0, b_table_sizes=[900, 900], a_immutable=False, tomb_frac=0.1)),
    ("account_history.timestamp", dict(n_a=300, b_table_sizes=[60, 90], a_immutable=True, dup_frac=0.2,
                                       tomb_frac=0.2, drop_tombstones=True, overlap=0.3)),
    ("transfers.amount", dict(n_a=1, b_table_sizes=[1], a_immutable=True, overlap=1.0)),
    ("accounts.id", dict(n_a=5, b_table_sizes=[], a_immutable=True)),
]


def test_compaction_parity_test_min_blocks(engine_small, oracle_lib):
    bs = 4096
    cases = []
    for name, kw in SMALL:
        base = trees.BY_NAME[name]
        # multi-block, multi-table outputs on 4 KiB blocks
        spec = trees.with_table_size(base, 5 * (bs - 256) // base.value_size + 3)
        cases.append((spec, kw))
    _compare(oracle_lib, engine_small, cases, bs)


def test_compaction_parity_production_blocks(engine, oracle_lib):
    bs = 1 << 20
    T = trees.BY_NAME
    cases = [
        (T["transfers.id"], dict(n_a=70_000, b_table_sizes=[262_080, 100_000], a_immutable=False, overlap=0.2)),
        (T["transfers.debit_account_id"], dict(n_a=80_000, b_table_sizes=[60_000], a_immutable=True,
                                                dup_frac=0.1, overlap=0.2, drop_tombstones=True)),
        (T["accounts.timestamp"], dict(n_a=60_000, b_table_sizes=[50_000, 9_000], a_immutable=True,
                                       dup_frac=0.5, tomb_frac=0.05, overlap=0.3, drop_tombstones=True)),
        (T["accounts.user_data_32"], dict(n_a=140_000, b_table_sizes=[70_000], a_immutable=True, dup_frac=0.1,
                                          overlap=0.1)),
    ]
    _compare(oracle_lib, engine, cases, bs, level_b=3)


def test_batch_of_mixed_trees_is_independent(engine_small, oracle_lib):
    # The same job alone and inside a batch gives identical bytes.
    bs = 4096
    spec = trees.with_table_size(trees.BY_NAME["transfers.code"], 1000)
    rng = np.random.default_rng(3)
    ji = workloads.make_job_inputs(spec, rng, n_a=1500, b_table_sizes=[400, 800], a_immutable=True,
                                   dup_frac=0.2, overlap=0.3)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, 2700, bs) + 1, rng, 5)
    alone, _ = gpu_run(engine_small, [ji], bs, [addrs])
    other = workloads.make_job_inputs(trees.with_table_size(trees.BY_NAME["accounts.id"], 900), rng, n_a=800,
                                      b_table_sizes=[300], a_immutable=False)
    oaddrs = workloads.addresses_for(workloads.worst_case_blocks(other.tree, 1100, bs) + 1, rng, 5)
    both, _ = gpu_run(engine_small, [other, ji], bs, [oaddrs, addrs])
    assert np.array_equal(alone[0][2], both[1][2])
    assert np.array_equal(alone[0][1], both[1][1])


@pytest.mark.parametrize("name", ["transfers.timestamp", "transfers.id", "accounts.ledger",
                                  "transfers.debit_account_id", "posted.timestamp", "account_history.timestamp"])
def test_sort_values_stable(engine, oracle_lib, name):
    """TableMemory.sort (table_memory.zig:140-154): stable, bit-exact vs the oracle."""
    spec = trees.BY_NAME[name]
    rng = np.random.default_rng(11)
    n = 70_001
    limbs = workloads.random_keys(spec, n, rng, field_max=300)
    limbs[0] = rng.integers(1, 5000, size=n, dtype=np.uint64)  # many equal keys: stability matters
    tomb = rng.random(n) < 0.1
    vals = workloads.values_from_keys(spec, limbs, tomb, rng)
    # Put the insertion order into bytes the key does not cover so that any
    # instability would show up in the output bytes.
    if spec.key_kind == 0:
        w = vals.view(np.uint64)
        w[:, (spec.timestamp_offset // 8 + 1) % (spec.value_size // 8)] = np.arange(n, dtype=np.uint64)
    elif spec.value_size == 32 and spec.key_kind == 1:
        vals.view(np.uint64)[:, 3] = np.arange(n, dtype=np.uint64)
    t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                        spec.value_count_max, 1 << 20)
    want = oracle_lib.sort_values(t, vals)
    buf = engine.upload(vals)
    engine.sort_values(spec, buf, n)
    got = buf.download(vals.nbytes).reshape(n, spec.value_size)
    assert np.array_equal(got, want)


def test_sort_values_already_sorted_is_noop(engine):
    spec = trees.BY_NAME["transfers.id"]
    rng = np.random.default_rng(12)
    limbs = workloads.unique_sorted_keys(spec, 5000, rng)
    vals = workloads.values_from_keys(spec, limbs, np.zeros(5000, dtype=bool), rng)
    buf = engine.upload(vals)
    engine.sort_values(spec, buf, 5000)
    assert np.array_equal(buf.download(vals.nbytes).reshape(5000, 32), vals)


def test_sort_values_low_limbs_in_order(engine, oracle_lib):
    """Tables already in order on their low key limbs, as a secondary index
    put in timestamp order is: the sort skips those limbs' passes
    (sort.hip k_sort_plan) and must still equal the oracle's stable sort.
    Cases: timestamps ascending (skip 1 limb); (field lo, timestamp) in order
    with the high field random and repeated keys (skip 2); an id whose low
    limb ascends (skip 1); and a composite u64 index with tombstones."""
    rng = np.random.default_rng(15)
    n = 50_001
    tables, wants = [], []

    def add(name, limbs, tomb=None):
        spec = trees.BY_NAME[name]
        vals = workloads.values_from_keys(spec, limbs, np.zeros(n, bool) if tomb is None else tomb, rng)
        t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                            spec.value_count_max, 1 << 20)
        wants.append(oracle_lib.sort_values(t, vals))
        tables.append((spec, engine.upload(vals, pad=16), n))

    ts = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(3)
    add("transfers.debit_account_id", [ts, rng.integers(1, 10_001, n, dtype=np.uint64), np.zeros(n, np.uint64)])
    lo = np.sort(rng.integers(0, 500, n, dtype=np.uint64))
    ts2 = rng.integers(1, 40, n, dtype=np.uint64)
    order = np.lexsort((ts2, lo))  # (lo, ts) ascending, duplicates kept
    add("transfers.credit_account_id", [ts2[order], lo[order], rng.integers(0, 3, n, dtype=np.uint64)])
    add("transfers.id", [np.arange(n, dtype=np.uint64), rng.integers(0, 1 << 40, n, dtype=np.uint64)])
    add("accounts.user_data_64", [ts, rng.integers(0, 1 << 62, n, dtype=np.uint64)], rng.random(n) < 0.1)
    engine.sort_values_batch(tables)
    engine.synchronize()
    for (spec, buf, _), want in zip(tables, wants):
        got = buf.download(n * spec.value_size).reshape(n, spec.value_size)
        assert np.array_equal(got, want), spec.name


def test_sort_truncated_top_bytes_and_rescue(engine, oracle_lib):
    """Tables with many varying key bytes are sorted on their top bytes only
    and each run of equal top bytes is ordered by k_sort_fixup (random u128
    and u64 fields put in timestamp order); a table whose top bytes cluster
    into runs too long to fix up is sorted again by k_sort_rescue. All equal
    to the oracle's stable sort, equal keys included."""
    rng = np.random.default_rng(16)
    n = 300_001
    ts = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(7)
    tables, wants = [], []

    def add(name, limbs):
        spec = trees.BY_NAME[name]
        vals = workloads.values_from_keys(spec, limbs, np.zeros(n, bool), rng)
        t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                            spec.value_count_max, 1 << 20)
        wants.append(oracle_lib.sort_values(t, vals))
        tables.append((spec, engine.upload(vals, pad=16), n))

    lo = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    hi = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    lo[: n // 3], hi[: n // 3] = lo[n // 3: 2 * (n // 3)], hi[n // 3: 2 * (n // 3)]  # repeated fields: runs ordered by timestamp
    add("transfers.user_data_128", [ts, lo, hi])
    add("transfers.user_data_64", [ts, rng.integers(0, 1 << 63, n, dtype=np.uint64)])
    # top four varying bytes take two values: runs of ~n/2 -> rescue
    c = rng.integers(1, 3, n, dtype=np.uint64)
    field = c * np.uint64(0x0101010100) + rng.integers(0, 256, n, dtype=np.uint64)
    add("transfers.user_data_64", [ts, field])
    engine.sort_values_batch(tables)
    engine.synchronize()
    for (spec, buf, _), want in zip(tables, wants):
        got = buf.download(n * spec.value_size).reshape(n, spec.value_size)
        assert np.array_equal(got, want), spec.name


def test_sort_values_many_passes(engine, oracle_lib):
    """Tables whose keys vary in more bytes than the direct pass launches
    cover (sort.hip kDirectPasses) and whose top bytes cluster, so the plan
    keeps every pass (no truncation): the passes past the direct ones run in
    k_sort_pass_rest, ordered by completion counters. Equal keys included;
    every table bit-exact vs the oracle's stable sort, in one batch."""
    rng = np.random.default_rng(21)
    n = 120_001
    tables, wants = [], []

    def add(name, limbs):
        spec = trees.BY_NAME[name]
        vals = workloads.values_from_keys(spec, limbs, rng.random(n) < 0.05, rng)
        t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                            spec.value_count_max, 1 << 20)
        wants.append(oracle_lib.sort_values(t, vals))
        tables.append((spec, engine.upload(vals, pad=16), n))

    def clustered(bits_random: int, top_bytes: int):
        x = rng.integers(0, 1 << bits_random, n, dtype=np.uint64)
        for b in range(top_bytes):  # each byte above takes one of two values
            x |= rng.integers(1, 3, n, dtype=np.uint64) << np.uint64(bits_random + 8 * b)
        return x
    # composite u128: 2 timestamp bytes + 5 field-lo bytes + 2 field-hi bytes = 9 passes
    add("transfers.user_data_128", [rng.integers(1, 1 << 16, n, dtype=np.uint64), clustered(16, 3),
                                    clustered(0, 2)])
    # object tree (u64 timestamp key): 8 varying bytes, top ones clustered
    add("transfers.timestamp", [clustered(24, 4) & np.uint64((1 << 63) - 1)])
    # id tree: 12 varying bytes
    add("transfers.id", [clustered(32, 4), clustered(8, 3)])
    engine.sort_values_batch([(spec, buf, m) for spec, buf, m in tables])
    engine.synchronize()
    for (spec, buf, m), want in zip(tables, wants):
        got = buf.download(m * spec.value_size).reshape(m, spec.value_size)
        assert np.array_equal(got, want), spec.name


@pytest.mark.parametrize("name", ["accounts.user_data_64", "transfers.debit_account_id"])
def test_sort_composite_key_cases(engine, oracle_lib, name):
    """composite_key.zig:88-124's cases on the device's key_from_value: the
    sort orders (1,100) < (1,101) < (2,99), and a tombstone (1, 100|bit) has
    the key of (1,100) (equal keys keep their put order)."""
    spec = trees.BY_NAME[name]
    bit = 1 << 63
    cases = [(2, 99), (1, 101), (1, 100 | bit), (1, 100), (1, 101 | bit)]
    vals = np.zeros((len(cases), spec.value_size), dtype=np.uint8)
    for i, (field, ts) in enumerate(cases):
        vals[i, :8].view(np.uint64)[0] = field
        vals[i, spec.timestamp_offset:spec.timestamp_offset + 8].view(np.uint64)[0] = np.uint64(ts)
    t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                        spec.value_count_max, 1 << 20)
    want = oracle_lib.sort_values(t, vals)
    order = [(int(w[:8].view(np.uint64)[0]), int(w[spec.timestamp_offset:spec.timestamp_offset + 8]
                                                  .view(np.uint64)[0])) for w in want]
    assert order == [(1, 100 | bit), (1, 100), (1, 101), (1, 101 | bit), (2, 99)]
    buf = engine.upload(vals, pad=16)
    engine.sort_values(spec, buf, len(cases))
    assert np.array_equal(buf.download(vals.nbytes).reshape(vals.shape), want)


def test_immutable_compaction_after_device_sort(engine, oracle_lib):
    """Bar end: sort the mutable table on the device, then compact it as the
    immutable table A (tree.zig:979-999 -> compaction.zig:483-559)."""
    from helpers import disk_image, run_oracle
    from tigerbeetle_amd.engine import Job, stage_blocks
    bs = 1 << 20
    spec = trees.BY_NAME["transfers.credit_account_id"]
    rng = np.random.default_rng(13)
    ji = workloads.make_job_inputs(spec, rng, n_a=50_000, b_table_sizes=[40_000], a_immutable=True,
                                   dup_frac=0.2, overlap=0.3, drop_tombstones=True, field_max=2000)
    shuffled = workloads.shuffle_for_memtable(ji.a_values, rng, spec)
    abuf = engine.upload(shuffled)
    engine.sort_values(spec, abuf, len(shuffled), sync=False)
    bbuf, segs_b = stage_blocks(engine, [workloads.split_blocks(t, 32760) for t in ji.b_tables], 32, bs)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, 90_000, bs) + 2, rng, 3)
    out = engine.alloc(len(addrs) * bs)
    batch = engine.submit([Job(spec, [(abuf.ptr, len(shuffled))], segs_b, True, True, 1, 7, 48, addrs, out)])
    batch.wait()
    r, infos = batch.result(0)
    blocks = out.download(r.block_count * bs).reshape(-1, bs)
    o = run_oracle(oracle_lib, ji, bs, addrs, cluster=7)
    assert r.block_count == len(o.blocks)
    for g, w in zip(blocks, o.blocks):
        assert np.array_equal(disk_image(g), disk_image(w))
    assert np.array_equal(infos, o.table_infos)


def test_sort_values_batch_of_memtables(engine, oracle_lib):
    """Bar end for many trees at once (tbc_sort_values_batch): every table
    bit-exact vs the oracle's stable sort; sorted, tiny and empty tables too."""
    rng = np.random.default_rng(14)
    names = ["transfers.debit_account_id", "transfers.timestamp", "accounts.ledger", "transfers.id",
             "posted.timestamp", "account_history.timestamp", "transfers.credit_account_id", "accounts.user_data_64"]
    sizes = [40_000, 9_000, 2049, 2048, 1, 3000, 0, 70_001]
    tables, bufs, wants = [], [], []
    for k, (name, n) in enumerate(zip(names, sizes)):
        spec = trees.BY_NAME[name]
        limbs = workloads.random_keys(spec, max(n, 1), rng, field_max=50)
        limbs[0] = rng.integers(1, 3000, size=max(n, 1), dtype=np.uint64)
        vals = workloads.values_from_keys(spec, limbs, rng.random(max(n, 1)) < 0.1, rng)[:n]
        if name == "transfers.timestamp":  # already sorted: must be left untouched
            vals = vals[np.argsort(workloads.keys_of(vals, spec)[0], kind="stable")]
        t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                            spec.value_count_max, 1 << 20)
        wants.append(oracle_lib.sort_values(t, vals) if n else vals)
        buf = engine.upload(vals, pad=16)
        bufs.append(buf)
        tables.append((spec, buf, n))
    engine.sort_values_batch(tables)
    engine.synchronize()
    for (spec, buf, n), want in zip(tables, wants):
        got = buf.download(n * spec.value_size).reshape(n, spec.value_size)
        assert np.array_equal(got, want), spec.name


def _bar_end_tables(oracle_lib, rng):
    """Tables of many trees (unsorted, in order, tiny, empty) and the oracle's
    stable sort of each."""
    names = ["transfers.debit_account_id", "transfers.timestamp", "accounts.ledger", "transfers.id",
             "posted.timestamp", "account_history.timestamp", "transfers.credit_account_id", "accounts.user_data_64"]
    sizes = [40_000, 9_000, 2049, 2048, 1, 3000, 0, 70_001]
    out = []
    for name, n in zip(names, sizes):
        spec = trees.BY_NAME[name]
        limbs = workloads.random_keys(spec, max(n, 1), rng, field_max=50)
        limbs[0] = rng.integers(1, 3000, size=max(n, 1), dtype=np.uint64)
        vals = workloads.values_from_keys(spec, limbs, rng.random(max(n, 1)) < 0.1, rng)[:n]
        if name == "transfers.timestamp":  # in key order
            vals = vals[np.argsort(workloads.keys_of(vals, spec)[0], kind="stable")]
        t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                            spec.value_count_max, 1 << 20)
        out.append((spec, vals, oracle_lib.sort_values(t, vals) if n else vals))
    return out


def test_sort_values_batch_out_of_place(engine, oracle_lib):
    """tbc_sort_job.values_out: every table sorted into its own output,
    bit-exact vs the oracle's stable sort (a table in order copied as is, a
    one-value table copied), the input left as put; an output overlapping its
    input is refused."""
    cases = _bar_end_tables(oracle_lib, np.random.default_rng(15))
    jobs, keep = [], []
    for spec, vals, want in cases:
        src = engine.upload(vals, pad=16)
        dst = engine.upload(np.full((max(len(vals), 1), spec.value_size), 0xEE, dtype=np.uint8), pad=16)
        keep.append((spec, vals, want, src, dst))
        jobs.append((spec, src, len(vals), dst.ptr))
    engine.sort_values_batch(jobs)
    engine.synchronize()
    for spec, vals, want, src, dst in keep:
        n = len(vals)
        assert np.array_equal(dst.download(n * spec.value_size).reshape(n, spec.value_size), want), spec.name
        assert np.array_equal(src.download(n * spec.value_size).reshape(n, spec.value_size), vals), spec.name
    spec, _, _, src, _ = keep[0]
    with pytest.raises(abi.TbcError):
        engine.sort_values_batch([(spec, src, 100, src.ptr + 16 * spec.value_size)])


def test_sort_values_batch_more_tiles_than_workgroups(engine, oracle_lib):
    """A batch of more 4,096-item tiles than the pass kernel keeps resident
    (3 x 256 workgroups): its passes take tiles by ticket; smaller batches
    give each tile its own workgroup (sort.hip sort_pass_tiles). Both
    orders, bit-exact vs the oracle's stable sort: random u128 ids (top-digit
    passes + run fixup) and a composite index with repeated accounts."""
    rng = np.random.default_rng(21)
    cases = []
    for name, n in (("transfers.id", 2_600_000), ("transfers.debit_account_id", 900_000)):
        spec = trees.BY_NAME[name]
        limbs = workloads.random_keys(spec, n, rng, field_max=None if name == "transfers.id" else 10_000)
        vals = workloads.values_from_keys(spec, limbs, rng.random(n) < 0.01, rng)
        t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                            spec.value_count_max, 1 << 20)
        cases.append((spec, vals, oracle_lib.sort_values(t, vals)))
    assert sum(-(-len(v) // 4096) for _, v, _ in cases) > 3 * 256
    jobs, keep = [], []
    for spec, vals, want in cases:
        src = engine.upload(vals, pad=16)
        dst = engine.upload(np.zeros_like(vals), pad=16)
        keep.append((spec, vals, want, dst))
        jobs.append((spec, src, len(vals), dst.ptr))
    engine.sort_values_batch(jobs)
    engine.synchronize()
    for spec, vals, want, dst in keep:
        n = len(vals)
        assert np.array_equal(dst.download(n * spec.value_size).reshape(n, spec.value_size), want), spec.name


def test_memtable_make_immutable(engine, oracle_lib):
    """tbc_memtable_make_immutable at a bar end: each mutable table's values
    become its immutable table's in key order (sorted out of place, or the
    buffers traded for a table put in order), the mutable tables empty and
    ready for the next bar's puts; a non-empty immutable table is refused."""
    from tigerbeetle_amd import Memtable
    cases = [c for c in _bar_end_tables(oracle_lib, np.random.default_rng(16)) if len(c[1])]
    pairs = []
    for spec, vals, want in cases:
        m, im = Memtable(engine, spec, capacity=len(vals) + 8), Memtable(engine, spec, capacity=len(vals) + 8)
        m.put(vals)
        pairs.append((m, im, spec.name == "transfers.timestamp"))
    Memtable.make_immutable(engine, pairs)
    for (spec, vals, want), (m, im, _) in zip(cases, pairs):
        ptr, n = im.values()
        assert n == len(vals) and m.values()[1] == 0
        got = np.zeros((n, spec.value_size), dtype=np.uint8)
        engine.synchronize()
        abi.check(abi.lib().tbc_copy_to_host(engine.handle, got.ctypes.data, ptr, got.nbytes), "copy")
        assert np.array_equal(got, want), spec.name
    # The next bar: puts into the emptied mutable tables, then its bar end
    # after the immutable tables were flushed (reset).
    spec, vals, want = cases[0]
    m, im, _ = pairs[0]
    m.put(vals[::-1].copy())
    with pytest.raises(abi.TbcError):  # the immutable table still holds the previous bar
        Memtable.make_immutable(engine, [(m, im, False)])
    im.reset()
    Memtable.make_immutable(engine, [(m, im, False)])
    ptr, n = im.values()
    got = np.zeros((n, spec.value_size), dtype=np.uint8)
    engine.synchronize()
    abi.check(abi.lib().tbc_copy_to_host(engine.handle, got.ctypes.data, ptr, got.nbytes), "copy")
    t = oracle_lib.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                        spec.value_count_max, 1 << 20)
    assert np.array_equal(got, oracle_lib.sort_values(t, vals[::-1].copy()))
    for m, im, _ in pairs:
        m.close()
        im.close()


def test_compaction_parity_throughput_regime(engine_small, oracle_lib):
    """More than 4,096 output data blocks in one batch switch the engine to
    its two-pass path (k_assemble, then chain-only k_data_blocks at 4 chains
    per SIMD); 4 KiB blocks reach that with small inputs."""
    bs = 4096
    T = trees.BY_NAME
    cases = []
    for i, name in enumerate(["transfers.id", "accounts.timestamp", "transfers.debit_account_id", "accounts.ledger",
                              "posted.timestamp", "transfers.id", "account_history.timestamp", "transfers.amount"]):
        base = T[name]
        spec = trees.with_table_size(base, 6 * (bs - 256) // base.value_size + 1)
        n = 125 * (bs - 256) // base.value_size  # 125 blocks of A, 4.5x that in all
        cases.append((spec, dict(n_a=n, b_table_sizes=[n // 2] * 7, a_immutable=i % 2 == 1, dup_frac=0.1 * (i % 2),
                                 tomb_frac=0.05 * (i % 3 != 2), drop_tombstones=i % 4 == 3, overlap=0.2)))
    # the batch must exceed the fused limit (2,048 chain waves = 4,096 blocks)
    total_blocks = sum(workloads.worst_case_blocks(s, kw["n_a"] * 9 // 2, bs) for s, kw in cases)
    assert total_blocks > 4096, total_blocks
    _compare(oracle_lib, engine_small, cases, bs)


def test_submit_rejects_broken_preconditions(engine_small):
    """The reference asserts (compaction.zig:307-318 reservation, 16-byte
    aligned values); the C ABI returns a status instead and runs nothing."""
    from tigerbeetle_amd.abi import TBC_ERR_CAPACITY, TBC_ERR_INVALID_ARGUMENT, TbcError
    from tigerbeetle_amd.engine import Job
    bs = 4096
    spec = trees.with_table_size(trees.BY_NAME["transfers.id"], 500)
    rng = np.random.default_rng(21)
    ji = workloads.make_job_inputs(spec, rng, n_a=300, b_table_sizes=[400], a_immutable=True, overlap=0.2)
    abuf = engine_small.upload(ji.a_values, pad=64)
    bbuf = engine_small.upload(ji.b_tables[0], pad=64)
    out = engine_small.alloc(64 * bs)
    few = np.arange(1, 3, dtype=np.uint64)  # 700 values need 6 data blocks + 2 index blocks
    with pytest.raises(TbcError) as e:
        engine_small.submit([Job(spec, [(abuf.ptr, 300)], [(bbuf.ptr, 400)], True, False, 1, 1, 48, few, out)])
    assert e.value.status == TBC_ERR_CAPACITY
    addrs = np.arange(1, 64, dtype=np.uint64)
    with pytest.raises(TbcError) as e:  # values must be 16-byte aligned
        engine_small.submit([Job(spec, [(abuf.ptr + 8, 300)], [(bbuf.ptr, 400)], True, False, 1, 1, 48, addrs, out)])
    assert e.value.status == TBC_ERR_INVALID_ARGUMENT
    with pytest.raises(TbcError) as e:  # an immutable table A is one segment
        engine_small.submit([Job(spec, [(abuf.ptr, 100), (abuf.ptr + 3200, 200)], [(bbuf.ptr, 400)], True, False, 1,
                                 1, 48, addrs, out)])
    assert e.value.status == TBC_ERR_INVALID_ARGUMENT
    # and the engine still works afterwards
    ok = engine_small.submit([Job(spec, [(abuf.ptr, 300)], [(bbuf.ptr, 400)], True, False, 1, 1, 48, addrs, out)])
    ok.wait()
    r, _ = ok.result(0)
    assert r.status == 0 and r.value_count > 0
    ok.release()


def test_blocks_validate_matches_grid_read_block_validate(engine_small, oracle_lib):
    """grid.read_block_validate (grid.zig:1059-1084) on the device: every
    output block of a compaction validates; each corruption is reported with
    the reference's result, in the reference's check order."""
    bs = 4096
    spec = trees.with_table_size(trees.BY_NAME["transfers.timestamp"], 100)
    rng = np.random.default_rng(31)
    ji = workloads.make_job_inputs(spec, rng, n_a=250, b_table_sizes=[80], a_immutable=True, dup_frac=0.1,
                                   overlap=0.2)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, 330, bs) + 2, rng, 40)
    (r, _, blocks), = gpu_run(engine_small, [ji], bs, [addrs])[0]
    n = r.block_count
    buf = engine_small.upload(blocks[:n])
    ptrs = [buf.ptr + i * bs for i in range(n)]
    cks = [int.from_bytes(b[0:16].tobytes(), "little") for b in blocks[:n]]
    adr = [int(b[224:232].view(np.uint64)[0]) for b in blocks[:n]]
    assert list(engine_small.validate_blocks(ptrs, cks, adr)) == [0] * n

    def corrupt(i, off, val, fix_header=False):
        img = blocks[i].copy()
        img[off] = val
        if fix_header:  # keep the header checksum valid (to reach the later checks)
            img[0:16] = np.frombuffer(oracle_lib.checksum(img[16:256].tobytes()).to_bytes(16, "little"), np.uint8)
        one = engine_small.upload(img)
        return int(engine_small.validate_blocks([one.ptr], [cks[i]], [adr[i]])[0])

    assert corrupt(0, 300, blocks[0][300] ^ 1) == 3          # body byte -> invalid_checksum_body
    assert corrupt(0, 232, blocks[0][232] ^ 1) == 1          # header byte -> invalid_checksum
    assert corrupt(0, 110, 19, fix_header=True) == 2         # command -> unexpected_command
    assert corrupt(0, 232, blocks[0][232] ^ 1, fix_header=True) == 4  # valid, but not the expected checksum
    wrong = engine_small.validate_blocks([ptrs[1]], [cks[1]], [adr[1] + 1])
    assert int(wrong[0]) == 5                                  # address mismatch


@pytest.mark.parametrize("bs", [4096, 1 << 20])
def test_heavy_dedup_jobs_pre_assembled(bs, engine, engine_small, oracle_lib):
    """Jobs with < 1/4 survivors (aegis.hip sparse_job: bodies by k_assemble
    before the fused chains) batched with dense ones; byte-exact vs oracle."""
    eng = engine if bs == 1 << 20 else engine_small
    rng = np.random.default_rng(0xDED0 + bs)
    def tree(name):
        t = trees.BY_NAME[name]
        return t if bs == 1 << 20 else trees.with_table_size(t, 3 * (bs - 256) // t.value_size + 5)
    acc = tree("accounts.timestamp")
    scale = 1 if bs == 1 << 20 else 40
    jobs = [
        workloads.make_job_inputs(acc, rng, n_a=200_000 // scale, b_table_sizes=[20_000 // scale],
                                  a_immutable=True, dup_frac=0.97, tomb_frac=0.02, overlap=0.5),
        workloads.make_job_inputs(acc, rng, n_a=5_000 // scale, b_table_sizes=[400_000 // scale],
                                  a_immutable=False, tomb_frac=0.9, drop_tombstones=True, overlap=0.0),
        workloads.make_job_inputs(tree("transfers.id"), rng, n_a=60_000 // scale,
                                  b_table_sizes=[70_000 // scale], a_immutable=True, dup_frac=0.05),
        # Secondary index, disk A, no tombstone drop: A's removes cancel 90 %
        # of B's puts (both vanish), so the job is sparse without dedup or
        # drop_tombstones (the host must still pre-assemble it).
        workloads.make_job_inputs(tree("transfers.debit_account_id"), rng, n_a=100_000 // scale,
                                  b_table_sizes=[100_000 // scale], a_immutable=False, overlap=0.9),
    ]
    addrs = [workloads.addresses_for(workloads.worst_case_blocks(ji.tree, len(ji.a_values) + sum(map(len, ji.b_tables)),
                                                                 bs) + 2, rng, 50 + 1000 * i) for i, ji in enumerate(jobs)]
    results, _ = gpu_run(eng, jobs, bs, addrs)
    for ji, a, (r, infos, blocks) in zip(jobs, addrs, results):
        o = run_oracle(oracle_lib, ji, bs, a)
        assert r.status == 0 and o.status == 0 and r.value_count == o.value_count
        assert len(blocks) == len(o.blocks)
        for g, w in zip(blocks, o.blocks):
            assert np.array_equal(disk_image(g), disk_image(w))
        assert np.array_equal(infos, o.table_infos)
    for k in (0, 3):  # the sparse path was taken
        nk = len(jobs[k].a_values) + sum(map(len, jobs[k].b_tables))
        assert results[k][0].value_count * 4 < nk, k
