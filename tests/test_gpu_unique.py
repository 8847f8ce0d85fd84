"""TBC_COMPACTION_UNIQUE_KEYS (include/tbc.h): the speculated block pass.

A job flagged UNIQUE_KEYS skips the merge pass: in the fused latency pass
each data block's producer merges its own positions while its AEGIS chain
absorbs them (aegis.hip produce_unique); in the pipelined pass the bodies
are merged tile by tile on the engine stream (merge.hip k_merge_unique) and
the chains run on a tail stream. Whether the speculation holds (no repeated key, no dropped
tombstone: every value survives) or breaks (then the batch's second phase
recomputes the job through the merge path), every output block's on-disk
image and every TableInfo must equal the oracle's restatement of
compaction.zig / table.zig, and tbc_batch_speculation must say which path
ran.
"""
import numpy as np
import pytest

from helpers import disk_image, gpu_run, run_oracle
from tigerbeetle_amd import abi, trees, workloads

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fused", "pipelined"])
def eng_small(request, engine_small, engine_small_pipe):
    """Both block passes of a speculated batch (engine.hip submit_impl): the
    fused latency pass (a batch alone), and the pipelined one (bodies merged
    by k_merge_unique on the engine stream, chains on a tail stream)."""
    return engine_small if request.param == "fused" else engine_small_pipe


@pytest.fixture(params=["fused", "pipelined"])
def eng(request, engine, engine_pipe):
    return engine if request.param == "fused" else engine_pipe

U = abi.COMPACTION_UNIQUE_KEYS
HELD, BROKEN, NONE = abi.SPECULATION_HELD, abi.SPECULATION_BROKEN, abi.SPECULATION_NONE


def _spec(name, block_size):
    """The tree at this block size: 4 KiB blocks get tables of ~5 data blocks
    (+3 values), so jobs span several output tables (test_gpu_parity.py)."""
    base = trees.BY_NAME[name]
    if block_size == 1 << 20:
        return base
    return trees.with_table_size(base, 5 * (block_size - 256) // base.value_size + 3)


def _run(oracle_lib, engine, cases, block_size, seed):
    """cases: (tree name, make_job_inputs kwargs, flags, expected speculation)."""
    rng = np.random.default_rng(seed)
    inputs, addrs, flags = [], [], []
    for name, kw, fl, _ in cases:
        spec = _spec(name, block_size)
        ji = workloads.make_job_inputs(spec, rng, **kw)
        n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
        addrs.append(workloads.addresses_for(workloads.worst_case_blocks(spec, n, block_size) + 3, rng,
                                             int(rng.integers(1, 1000)), 0.1))
        inputs.append(ji)
        flags.append(fl)
    outcome = []
    results, _ = gpu_run(engine, inputs, block_size, addrs, flags=flags, speculation=outcome)
    for (name, _, _, want), ji, a, (r, infos, blocks), got in zip(cases, inputs, addrs, results, outcome):
        o = run_oracle(oracle_lib, ji, block_size, a)
        assert o.status == 0 and r.status == 0, name
        assert got == want, (name, got, want)
        assert r.value_count == o.value_count and r.block_count == len(o.blocks), name
        for g, w in zip(blocks, o.blocks):
            assert np.array_equal(disk_image(g), disk_image(w)), name
        assert np.array_equal(infos, o.table_infos), name


UNIQUE_TREES = ["transfers.id", "transfers.timestamp", "transfers.debit_account_id", "transfers.ledger",
                "account_history.timestamp"]


@pytest.mark.parametrize("name", UNIQUE_TREES)
def test_unique_held_small_blocks(oracle_lib, eng_small, name):
    """Unique keys (disk A, immutable A, A only, B only): speculation holds."""
    cases = [
        (name, dict(n_a=3000, b_table_sizes=[2000, 1500, 900], a_immutable=False, overlap=0.0), U, HELD),
        (name, dict(n_a=2500, b_table_sizes=[4000], a_immutable=True, overlap=0.0), U, HELD),
        (name, dict(n_a=1700, b_table_sizes=[], a_immutable=True, overlap=0.0), U, HELD),
        (name, dict(n_a=0, b_table_sizes=[777, 123], a_immutable=False, overlap=0.0), U, HELD),
        (name, dict(n_a=1, b_table_sizes=[1], a_immutable=False, overlap=0.0), U, HELD),
    ]
    _run(oracle_lib, eng_small, cases, 4096, seed=11)


@pytest.mark.parametrize("name", ["transfers.id", "transfers.timestamp", "transfers.debit_account_id",
                                  "accounts.ledger"])
def test_unique_broken_small_blocks(oracle_lib, eng_small, name):
    """Repeated keys (A/B overlap, immutable duplicates, secondary put/remove
    pairs) and dropped tombstones break the speculation; the recomputation
    must give the merge path's blocks, beside jobs whose speculation holds and
    jobs not speculated at all."""
    secondary = trees.BY_NAME[name].usage == abi.USAGE_SECONDARY_INDEX
    cases = [
        (name, dict(n_a=3000, b_table_sizes=[2000, 1500], a_immutable=False, overlap=0.05), U, BROKEN),
        (name, dict(n_a=2600, b_table_sizes=[1800], a_immutable=True, overlap=0.0, dup_frac=0.01), U, BROKEN),
        (name, dict(n_a=2000, b_table_sizes=[2000], a_immutable=False, overlap=0.0), U, HELD),
        (name, dict(n_a=2000, b_table_sizes=[2000], a_immutable=False, overlap=0.1), 0, NONE),
    ]
    if not secondary:
        cases.append((name, dict(n_a=2500, b_table_sizes=[900], a_immutable=False, overlap=0.0, tomb_frac=0.01,
                                 drop_tombstones=True), U, BROKEN))
        # tombstones kept (not the last level): speculation holds
        cases.append((name, dict(n_a=2500, b_table_sizes=[900], a_immutable=False, overlap=0.0, tomb_frac=0.05),
                      U, HELD))
    _run(oracle_lib, eng_small, cases, 4096, seed=12)


@pytest.mark.parametrize("name", ["transfers.id", "transfers.debit_account_id"])
def test_unique_most_significant_limb_ties(oracle_lib, eng_small, name):
    """Keys whose most significant 64 bits take only three values (field_max):
    the pipelined merge keeps only those bits in LDS, so nearly every
    comparison falls back to the full keys read from the values. Held and
    broken speculations must still give the merge path's blocks."""
    cases = [
        (name, dict(n_a=3000, b_table_sizes=[2000, 1500], a_immutable=False, overlap=0.0, field_max=3), U, HELD),
        (name, dict(n_a=2500, b_table_sizes=[2500], a_immutable=True, overlap=0.0, field_max=3), U, HELD),
        (name, dict(n_a=3000, b_table_sizes=[2000], a_immutable=False, overlap=0.02, field_max=3), U, BROKEN),
    ]
    _run(oracle_lib, eng_small, cases, 4096, seed=14)


def _repeat_at_block_start(spec, vcm, block: int, first_in_a: bool, seed: int) -> workloads.JobInputs:
    """Inputs whose merged order (A-first tie break) has exactly one repeated
    key, at merged positions (block*vcm - 1, block*vcm): the last value of data
    block `block - 1` and the first of data block `block` under the
    speculation's layout. One of the pair is in A and the other in B
    (`first_in_a` says which comes first), so both streams stay strictly
    increasing and only the cross-stream check at a producer's first
    position can see the repeat."""
    rng = np.random.default_rng(seed)
    n = 6 * vcm + 17
    limbs = workloads.unique_sorted_keys(spec, n, rng)
    vals = workloads.values_from_keys(spec, limbs, np.zeros(n, dtype=bool), rng)
    k = block * vcm                           # first merged position of `block`
    in_a = rng.random(n) < 0.5
    in_a[k - 1], in_a[k] = first_in_a, not first_in_a
    dup = vals[k].copy()
    dup[:16] = vals[k - 1][:16]               # id (the key) of the position before
    vals[k] = dup
    a, b = vals[in_a], vals[~in_a]
    # B as tables of whole blocks (a table holds 5 data blocks + 3 values at 4 KiB)
    tmax = spec.value_count_max
    return workloads.JobInputs(spec, a, False, [b[i:i + tmax] for i in range(0, len(b), tmax)], False)


@pytest.mark.parametrize("block,first_in_a", [(1, True), (1, False), (2, True), (4, False)])
def test_unique_one_repeat_at_a_block_boundary(oracle_lib, eng_small, block, first_in_a):
    """A single repeated key exactly where a data block starts: the check that
    crosses producers (a producer's first value against its predecessor in
    the previous block) must break the speculation, and the recomputed blocks
    must be the reference's. Constructed, never skipped."""
    spec = _spec("transfers.id", 4096)
    vcm = eng_small.layout(spec).block_value_count_max
    ji = _repeat_at_block_start(spec, vcm, block, first_in_a, seed=3 + block)
    n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
    rng = np.random.default_rng(5)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n, 4096) + 3, rng, 5)
    outcome = []
    (res,), _ = gpu_run(eng_small, [ji], 4096, [addrs], flags=U, speculation=outcome)
    r, infos, blocks = res
    o = run_oracle(oracle_lib, ji, 4096, addrs)
    assert o.status == 0 and r.status == 0
    assert o.value_count == n - 1             # the A copy of the repeated key wins, the B copy is dropped
    assert outcome == [BROKEN]
    assert r.value_count == o.value_count and r.block_count == len(o.blocks)
    for g, w in zip(blocks, o.blocks):
        assert np.array_equal(disk_image(g), disk_image(w))
    assert np.array_equal(infos, o.table_infos)


def test_unique_no_repeat_at_block_starts_holds(oracle_lib, eng_small):
    """The same construction without the repeat (A/B alternate across every
    block start): the speculation holds."""
    spec = _spec("transfers.id", 4096)
    vcm = eng_small.layout(spec).block_value_count_max
    rng = np.random.default_rng(9)
    n = 6 * vcm + 17
    limbs = workloads.unique_sorted_keys(spec, n, rng)
    vals = workloads.values_from_keys(spec, limbs, np.zeros(n, dtype=bool), rng)
    in_a = np.arange(n) % 2 == 0
    tmax = spec.value_count_max
    b = vals[~in_a]
    ji = workloads.JobInputs(spec, vals[in_a], False, [b[i:i + tmax] for i in range(0, len(b), tmax)], False)
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n, 4096) + 3, rng, 5)
    outcome = []
    (res,), _ = gpu_run(eng_small, [ji], 4096, [addrs], flags=U, speculation=outcome)
    r, infos, blocks = res
    o = run_oracle(oracle_lib, ji, 4096, addrs)
    assert outcome == [HELD] and r.block_count == len(o.blocks)
    for g, w in zip(blocks, o.blocks):
        assert np.array_equal(disk_image(g), disk_image(w))
    assert np.array_equal(infos, o.table_infos)


def test_unique_config2_shape(oracle_lib, eng):
    """1 MiB blocks, BASELINE config 2's job shape scaled down (disk A + 8 B
    tables of the transfers.id tree), held; plus one broken job in the batch."""
    name = "transfers.id"
    cases = [(name, dict(n_a=120_000, b_table_sizes=[40_000] * 8, a_immutable=False, overlap=0.0), U, HELD)
             for _ in range(3)]
    cases.append((name, dict(n_a=90_000, b_table_sizes=[30_000] * 4, a_immutable=False, overlap=0.001), U, BROKEN))
    _run(oracle_lib, eng, cases, 1 << 20, seed=21)
