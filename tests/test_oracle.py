"""CPU tests: the oracle against the reference's own known-answer tests, and
the oracle's chunked compaction loop against a global restatement.

Reference KATs: src/vsr/checksum.zig:94-112 (test vectors), :146-195
(checksum stability), src/lsm/composite_key.zig:88-124,
src/lsm/table_memory.zig:190-220.
"""
import numpy as np
import pytest

import zig_prng
from helpers import data_values_from_blocks, model_merge, oracle_tree, run_oracle
from tigerbeetle_amd import trees, workloads
from tigerbeetle_amd.abi import KEY_COMPOSITE_U64, KEY_COMPOSITE_U128


def bswap128(x):
    return int.from_bytes(x.to_bytes(16, "big"), "little")


@pytest.mark.parametrize("portable", [False, True])
def test_checksum_test_vectors(oracle_lib, portable):
    # checksum.zig:100-108
    assert oracle_lib.checksum(bytes(16), portable) == bswap128(0xF72AD48DD05DD1656133101CD4BE3A26)
    assert oracle_lib.checksum(b"", portable) == bswap128(0x83CC600DC4E3E7E62D4055826174F149)
    # checksum.zig:54 comptime value for the empty message
    assert oracle_lib.checksum(b"", portable) == 0x49F174618255402DE6E7E3C40D60CC83


@pytest.mark.parametrize("portable", [False, True])
def test_checksum_stability(oracle_lib, portable):
    msgs = zig_prng.stability_messages()
    assert len(msgs) == 896
    cases = [oracle_lib.checksum(m, portable) for m in msgs]
    assert len(set(cases)) == 896 and 0 not in cases and (1 << 128) - 1 not in cases
    blob = b"".join(c.to_bytes(16, "little") for c in cases)
    assert oracle_lib.checksum(blob, portable) == zig_prng.STABILITY_HASH


def test_checksum_simple_fuzzing(oracle_lib):
    # checksum.zig:114-143 (pure function; a changed byte changes the checksum)
    rng = np.random.default_rng(42)
    for _ in range(50):
        n = int(rng.integers(1, 1 << 16))
        m = bytearray(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        c = oracle_lib.checksum(bytes(m))
        assert c == oracle_lib.checksum(bytes(m))
        m[int(rng.integers(0, n))] ^= 1
        assert oracle_lib.checksum(bytes(m)) != c
        assert oracle_lib.checksum(bytes(m), True) == oracle_lib.checksum(bytes(m), False)


@pytest.mark.parametrize("kind", [KEY_COMPOSITE_U64, KEY_COMPOSITE_U128])
def test_composite_key(oracle_lib, kind):
    # composite_key.zig:88-124 (composite_key_test, all four blocks) through
    # the oracle's key_from_value / tombstone / tombstone_from_key.
    import ctypes
    spec = next(t for t in trees.TREES if t.key_kind == kind)
    t = oracle_tree(oracle_lib, spec, trees.BLOCK_SIZE)
    L = oracle_lib.lib()

    def value(field, ts):
        v = np.zeros(spec.value_size, dtype=np.uint8)
        v[:8].view(np.uint64)[0] = field
        v[spec.timestamp_offset:spec.timestamp_offset + 8].view(np.uint64)[0] = np.uint64(ts)
        return v

    def key(v):
        out = (ctypes.c_uint64 * 4)()
        L.tbo_key(ctypes.byref(t), v.ctypes.data, out)
        return sum(int(out[i]) << (64 * i) for i in range(4))

    bit = 1 << 63
    assert key(value(1, 100)) < key(value(1, 101))                    # :89-93
    assert key(value(1, 100)) < key(value(2, 99))                     # :95-99
    assert key(value(1, 100 | bit)) == key(value(1, 100))             # :101-111
    k = key(value(1, 100))                                            # :113-118
    limbs = (ctypes.c_uint64 * 4)(*[(k >> (64 * i)) & ((1 << 64) - 1) for i in range(4)])
    tomb = np.zeros(spec.value_size, dtype=np.uint8)
    assert L.tbo_tombstone_from_key(ctypes.byref(t), limbs, tomb.ctypes.data) == 0
    assert L.tbo_tombstone(ctypes.byref(t), tomb.ctypes.data) == 1
    assert int(tomb[spec.timestamp_offset:spec.timestamp_offset + 8].view(np.uint64)[0]) == 100 | bit
    assert int(tomb[:8].view(np.uint64)[0]) == 1 and key(tomb) == k
    # tombstone_from_key asserts the key's timestamp has no tombstone bit (:67)
    bad = (ctypes.c_uint64 * 4)(100 | bit, 1, 0, 0)
    assert L.tbo_tombstone_from_key(ctypes.byref(t), bad, tomb.ctypes.data) != 0


def test_tree_layouts_match_survey(oracle_lib):
    # SURVEY.md §8(a) table, derived from table.zig:107-129 / schema.zig:119-157.
    expect = {7: (8190, 64, 3840), 19: (8190, 32, 2048), 21: (4095, 64, 3840), 20: (65520, 4, 480),
              1: (32760, 8, 832), 8: (32760, 8, 832), 9: (32760, 8, 1088), 3: (65520, 4, 544)}
    for tid, (vcm, dbcm, isize) in expect.items():
        spec = trees.BY_ID[tid]
        t = oracle_tree(oracle_lib, spec, trees.BLOCK_SIZE)
        assert (t.block_value_count_max, t.data_block_count_max, t.index_size) == (vcm, dbcm, isize)
        lay = spec.layout()
        assert (lay["block_value_count_max"], lay["data_block_count_max"], lay["index_size"]) == (vcm, dbcm, isize)


def test_table_memory_sort_stable(oracle_lib):
    # table_memory.zig:190-220 plus stability ("last put wins", tree_fuzz.zig:442-468).
    spec = trees.BY_NAME["transfers.debit_account_id"]
    t = oracle_tree(oracle_lib, spec, trees.BLOCK_SIZE)
    rng = np.random.default_rng(7)
    limbs = workloads.random_keys(spec, 5000, rng, field_max=50)
    limbs[0] = rng.integers(1, 40, size=5000, dtype=np.uint64)
    vals = workloads.values_from_keys(spec, limbs, np.zeros(5000, dtype=bool), rng)
    vals.view(np.uint64)[:, 3] = np.arange(5000, dtype=np.uint64)  # insertion order in padding
    out = oracle_lib.sort_values(t, vals)
    keys = workloads.keys_of(out, spec)
    order = workloads.sort_keys(workloads.keys_of(vals, spec))
    assert np.array_equal(out, vals[order])
    k = np.stack(keys[::-1], axis=1)
    assert all(tuple(k[i]) <= tuple(k[i + 1]) for i in range(len(k) - 1))


CASES = [
    # (tree name, n_a, b_table_sizes, a_immutable, dup_frac, tomb_frac, drop, overlap)
    ("transfers.id", 700, [300, 500], False, 0.0, 0.0, False, 0.3),
    ("transfers.id", 900, [400], True, 0.2, 0.1, True, 0.5),
    ("transfers.timestamp", 400, [100, 150, 90], True, 0.3, 0.2, False, 0.4),
    ("transfers.timestamp", 400, [], False, 0.0, 0.3, True, 0.0),
    ("transfers.debit_account_id", 800, [300, 200], True, 0.4, 0.0, True, 0.3),
    ("accounts.ledger", 600, [500], True, 0.3, 0.0, False, 0.5),
    ("posted.timestamp", 0, [300, 300], False, 0.0, 0.1, False, 0.0),
    ("account_history.timestamp", 120, [60, 90], True, 0.2, 0.2, True, 0.3),
]


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_global_model(oracle_lib, case):
    name, n_a, bsizes, imm, dup, tomb, drop, overlap = case
    # test_min-shaped blocks (4 KiB) with multi-block tables so output spans tables.
    spec = trees.with_table_size(trees.BY_NAME[name], 4 * (4096 - 256) // trees.BY_NAME[name].value_size + 7)
    rng = np.random.default_rng(CASES.index(case) + 1000)
    ji = workloads.make_job_inputs(spec, rng, n_a=n_a, b_table_sizes=bsizes, a_immutable=imm, overlap=overlap,
                                   dup_frac=dup, tomb_frac=tomb, drop_tombstones=drop)
    bs = 4096
    addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n_a + sum(bsizes), bs) + 4, rng, 10, 0.2)
    r = run_oracle(oracle_lib, ji, bs, addrs)
    assert r.status == 0
    got = data_values_from_blocks(r.blocks, spec.value_size)
    want = model_merge(ji)
    assert np.array_equal(got, want)
    assert r.value_count == len(want)
    # Every block's header and body checksums verify (grid.zig:1059-1084).
    for blk in r.blocks:
        size = int(blk[96:100].view(np.uint32)[0])
        assert oracle_lib.checksum(blk[256:size].tobytes()) == int.from_bytes(blk[32:48].tobytes(), "little")
        assert oracle_lib.checksum(blk[16:256].tobytes()) == int.from_bytes(blk[0:16].tobytes(), "little")
        assert int(blk[224:232].view(np.uint64)[0]) in set(int(a) for a in addrs)
