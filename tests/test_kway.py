"""CPU: the k-way merge oracle (oracle.kway_merge, a line-by-line restatement
of KWayMergeIteratorType, src/lsm/k_way_merge.zig:8-205) against the
reference's own unit vectors (:396-461) and its fuzz expectation (:288-358:
sort by key, higher stream first on ties, keep the first of each key)."""
import numpy as np
import pytest

from oracle import oracle


def _merge(streams, descending=False):
    return oracle.kway_merge([[(k, v) for k in s] for v, s in enumerate(streams)], descending)


def test_reference_unit_vectors():
    # k_way_merge.zig:397-420 (k = 1)
    assert _merge([[0, 3, 4, 8]]) == [(0, 0), (3, 0), (4, 0), (8, 0)]
    assert _merge([[8, 4, 3, 0]], True) == [(8, 0), (4, 0), (3, 0), (0, 0)]
    # :421-440 (k = 3, ascending)
    assert _merge([[0, 3, 4, 8, 11], [2, 11, 12, 13, 15], [1, 2, 11]]) == [
        (0, 0), (1, 2), (2, 2), (3, 0), (4, 0), (8, 0), (11, 2), (12, 1), (13, 1), (15, 1)]
    # :441-460 (k = 3, descending)
    assert _merge([[11, 8, 4, 3, 0], [15, 13, 12, 11, 2], [11, 2, 1]], True) == [
        (15, 1), (13, 1), (12, 1), (11, 2), (8, 0), (4, 0), (3, 0), (2, 2), (1, 2), (0, 0)]


def _fuzz_streams(rng, k, count_max):
    streams = []
    for _ in range(k):
        r = rng.integers(0, 100)  # fuzz_stream_len, :360-366
        n = 0 if r < 5 else count_max if r < 10 else int(rng.integers(0, count_max + 1))
        key_max = int(rng.integers(512, 1024))
        if rng.integers(0, 100) < 5:  # fuzz_stream_keys, :368-380
            keys = np.full(n, int(rng.integers(0, 1 << 32)), dtype=np.uint64)
        else:
            keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64)
        streams.append(sorted(int(x) % key_max for x in keys))
    return streams


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_against_reference_expectation(seed):
    rng = np.random.default_rng(seed)
    for k in range(0, 12):
        streams = _fuzz_streams(rng, k, 128)
        flat = sorted(((key, v) for v, s in enumerate(streams) for key in s), key=lambda x: (x[0], -x[1]))
        expect, prev = [], None
        for key, v in flat:
            if key != prev:
                expect.append((key, v))
                prev = key
        assert _merge(streams) == expect
        assert _merge([s[::-1] for s in streams], True) == expect[::-1]


def test_elementwise_formulation_matches_heap():
    # The GPU's formulation (kway.hip): (s, i) is emitted iff first of its run
    # in s and no higher stream has the key; position = emitted keys before it.
    rng = np.random.default_rng(7)
    for _ in range(30):
        streams = _fuzz_streams(rng, int(rng.integers(1, 9)), 64)
        out = {}
        for s, st in enumerate(streams):
            for i, key in enumerate(st):
                first = i == 0 or st[i - 1] != key
                if first and not any(key in streams[t] for t in range(s + 1, len(streams))):
                    out[key] = (key, s)
        assert [out[key] for key in sorted(out)] == _merge(streams)
