"""GPU: tbc_kway_merge (the scan path's k-way merge, kway.hip) against the
oracle's restatement of KWayMergeIteratorType (k_way_merge.zig:8-205), byte
for byte, for every key kind, both directions, with repeated keys inside a
stream, keys shared across streams, empty streams; plus the reference's own
unit vectors (:396-461) carried in a timestamp-keyed tree."""
import numpy as np
import pytest

from oracle import oracle
from tigerbeetle_amd import trees, workloads

pytestmark = pytest.mark.gpu

TREES = ["transfers.timestamp", "transfers.id", "transfers.ledger", "transfers.debit_account_id"]


def _key_tuples(values, spec):
    limbs = workloads.keys_of(values, spec)
    return [tuple(int(l[i]) for l in reversed(limbs)) for i in range(len(values))]


def _run(engine, spec, streams, descending):
    vs = spec.value_size
    bufs = [engine.upload(s) if len(s) else None for s in streams]
    segs = [(b.ptr if b else 0, len(s)) for b, s in zip(bufs, streams)]
    total = sum(len(s) for s in streams)
    out = engine.alloc(max(1, total) * vs)
    n = engine.kway_merge(spec, segs, out if total else None, descending)
    return out.download(n * vs).reshape(-1, vs) if n else np.zeros((0, vs), np.uint8)


def _expect(spec, streams, descending):
    merged = oracle.kway_merge([list(zip(_key_tuples(s, spec), [bytes(v) for v in s])) for s in streams],
                               descending)
    return b"".join(v for _, v in merged)


@pytest.mark.parametrize("name", TREES)
@pytest.mark.parametrize("descending", [False, True])
def test_kway_matches_oracle(engine, name, descending):
    spec = trees.BY_NAME[name]
    rng = np.random.default_rng(len(name) * 2 + descending)
    for k, n_max, universe in [(1, 3000, 2000), (3, 20000, 30000), (9, 20000, 60000), (16, 800, 300)]:
        limbs = workloads.unique_sorted_keys(spec, universe, rng)
        streams = []
        for s in range(k):
            n = 0 if rng.random() < 0.1 else int(rng.integers(1, n_max))
            idx = np.sort(rng.integers(0, universe, size=n))  # repeats inside a stream
            v = workloads.values_from_keys(spec, [l[idx] for l in limbs], np.zeros(n, bool), rng)
            streams.append(v[::-1].copy() if descending else v)
        got = _run(engine, spec, streams, descending)
        assert got.tobytes() == _expect(spec, streams, descending), (k, n_max)


def test_kway_reference_unit_vectors(engine):
    # k_way_merge.zig:421-460 with Value {key, version} as a 16-byte object
    # value: timestamp = key, version in the second word.
    spec = trees.with_table_size(trees.BY_NAME["transfers.timestamp"], 1000)
    spec = trees.TreeSpec("kway.test", 250, spec.key_kind, spec.usage, 16, 0, 1000)

    def values(keys, version):
        v = np.zeros((len(keys), 2), np.uint64)
        v[:, 0], v[:, 1] = keys, version
        return v.view(np.uint8).reshape(-1, 16)

    for desc, streams, expect in [
        (False, [[0, 3, 4, 8, 11], [2, 11, 12, 13, 15], [1, 2, 11]],
         [(0, 0), (1, 2), (2, 2), (3, 0), (4, 0), (8, 0), (11, 2), (12, 1), (13, 1), (15, 1)]),
        (True, [[11, 8, 4, 3, 0], [15, 13, 12, 11, 2], [11, 2, 1]],
         [(15, 1), (13, 1), (12, 1), (11, 2), (8, 0), (4, 0), (3, 0), (2, 2), (1, 2), (0, 0)]),
    ]:
        got = _run(engine, spec, [values(s, i) for i, s in enumerate(streams)], desc)
        assert [tuple(int(x) for x in r) for r in got.view(np.uint64).reshape(-1, 2)] == expect


def test_kway_empty(engine):
    spec = trees.BY_NAME["transfers.id"]
    assert len(_run(engine, spec, [], False)) == 0
    assert len(_run(engine, spec, [np.zeros((0, 32), np.uint8)] * 3, True)) == 0


def test_kway_async_handles(engine):
    """tbc_kway_merge_submit returns at once; two merges in flight, polled to
    completion, give the blocking call's bytes and counts."""
    spec = trees.BY_NAME["transfers.id"]
    rng = np.random.default_rng(7)
    limbs = workloads.unique_sorted_keys(spec, 50_000, rng)
    streams = []
    for _ in range(5):
        idx = np.sort(rng.integers(0, 50_000, size=int(rng.integers(1000, 20_000))))
        streams.append(workloads.values_from_keys(spec, [l[idx] for l in limbs], np.zeros(len(idx), bool), rng))
    bufs = [engine.upload(s) for s in streams]
    segs = [(b.ptr, len(s)) for b, s in zip(bufs, streams)]
    total = sum(len(s) for s in streams)
    outs = [engine.alloc(total * 32) for _ in range(2)]
    hs = [engine.kway_merge_submit(spec, segs, outs[0]), engine.kway_merge_submit(spec, segs[::-1], outs[1])]
    import time
    deadline = time.time() + 30
    while not all(h.poll() for h in hs):
        assert time.time() < deadline
    counts = [h.count() for h in hs]
    for h in hs[::-1]:
        h.release()
    want0, want1 = _run(engine, spec, streams, False), _run(engine, spec, streams[::-1], False)
    assert counts == [len(want0), len(want1)]
    assert np.array_equal(outs[0].download(counts[0] * 32).reshape(-1, 32), want0)
    assert np.array_equal(outs[1].download(counts[1] * 32).reshape(-1, 32), want1)
