"""Memtable sort alone: the bar-end sort batch of config 3 or 4 (every
unsorted memtable of the job set), timed over repeated land + sort rounds.

  python tools/sort_probe.py [--config 3] [--reps 20]

Prints one JSON line: ms per sort batch (land copies subtracted), items,
bytes, and whether the last round's output equals numpy's stable sort.
Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from tigerbeetle_amd import Engine, configs, workloads

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--jobs", type=int, default=0)
args = ap.parse_args()

njobs = args.jobs or configs.DEFAULT_JOBS[args.config]
eng = Engine(device=0, block_size=1 << 20)
tables, landings, host = [], [], []
for gid in range(njobs):
    js = configs.GENERATORS[args.config](gid)
    if not (js.a_immutable and js.a_unsorted):
        continue
    buf, pristine = eng.upload(js.a), eng.upload(js.a)
    tables.append((js.tree, buf, len(js.a)))
    landings.append((buf.ptr, pristine.ptr, js.a.nbytes, buf, pristine))
    host.append(js)


def land():
    eng.copy_device_batch([(dst, src, n) for dst, src, n, _, _ in landings])


def timed(fn, reps):
    fn()
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    eng.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


t_land = timed(land, args.reps)
t_both = timed(lambda: (land(), eng.sort_values_batch(tables)), args.reps)
ok = True
for js, (tree, buf, n) in zip(host, tables):
    got = buf.download(n * tree.value_size).reshape(n, tree.value_size)
    want = js.a[workloads.sort_keys(workloads.keys_of(js.a, tree))]
    ok &= bool(np.array_equal(got, want))
items = sum(n for _, _, n in tables)
nbytes = sum(n * t.value_size for t, _, n in tables)
print(json.dumps({"config": args.config, "tables": len(tables), "items": items, "bytes": nbytes,
                  "land_ms": round(t_land, 4), "sort_ms": round(t_both - t_land, 4), "bit_exact": ok}), flush=True)
eng.close()
