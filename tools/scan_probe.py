"""Scan-path k-way merge throughput on one GPU (tbc_kway_merge).

    python tools/scan_probe.py [--streams 8] [--per-stream 2000000] [--tree transfers.id]

k sorted streams of Values resident in HBM (repeated and shared keys), merged
ascending; prints one JSON line with the wall time per merge (the call is
synchronous) and the algorithmic bytes: every input value read by the flag
kernel and the emitted ones written by the scatter (key probes excluded)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tigerbeetle_amd import Engine, trees, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--per-stream", type=int, default=2_000_000)
    ap.add_argument("--tree", default="transfers.id")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    spec = trees.BY_NAME[a.tree]
    rng = np.random.default_rng(1)
    universe = a.streams * a.per_stream
    limbs = workloads.unique_sorted_keys(spec, universe, rng)
    with Engine(device=0) as eng:
        bufs, segs = [], []
        for _ in range(a.streams):
            idx = np.sort(rng.choice(universe, size=a.per_stream, replace=False))
            v = workloads.values_from_keys(spec, [l[idx] for l in limbs], np.zeros(len(idx), bool), rng)
            b = eng.upload(v)
            bufs.append(b)
            segs.append((b.ptr, len(v)))
        total = a.streams * a.per_stream
        out = eng.alloc(total * spec.value_size)
        n = eng.kway_merge(spec, segs, out)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            n = eng.kway_merge(spec, segs, out)
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        alg = (total + n) * spec.value_size
        print(json.dumps({"probe": "kway_merge", "tree": a.tree, "streams": a.streams, "values_in": total,
                          "values_out": n, "ms": round(t * 1e3, 3), "alg_bytes": alg,
                          "alg_GBps": round(alg / t / 1e9, 1), "frac_of_8TBps": round(alg / t / 8e12, 4)}))


if __name__ == "__main__":
    main()
