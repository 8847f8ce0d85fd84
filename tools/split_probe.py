"""Cost of the key-range split path on one GPU (tigerbeetle_amd/split.py).

    python tools/split_probe.py [--reps 5]

One config-2 compaction (transfers.id, 1 disk A table + 8 B tables, 2.36 M
values) run directly and through compact_split with a world of one (phase 1
values-only + phase 2 re-blocking, no exchange), checking that both write the
same blocks. Prints one JSON line of median wall times per job."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tigerbeetle_amd import Engine, configs, split, workloads  # noqa: E402
from tigerbeetle_amd.engine import Job, stage_blocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    js = configs.config2_job(0)
    spec, bs = js.tree, 1 << 20
    with Engine(device=0, block_size=bs) as eng:
        vcm = eng.layout(spec).block_value_count_max
        abuf, segs_a = stage_blocks(eng, [workloads.split_blocks(js.a, vcm)], spec.value_size, bs)
        bbuf, segs_b = stage_blocks(eng, [workloads.split_blocks(t, vcm) for t in js.b_tables], spec.value_size, bs)
        n = js.input_values
        addrs = np.arange(1, workloads.worst_case_blocks(spec, n, bs) + 1, dtype=np.uint64)
        out = eng.alloc(len(addrs) * bs)
        job = Job(spec, segs_a, segs_b, False, False, 1, 7, 48, addrs, out)

        def direct():
            b = eng.submit([job])
            b.wait()
            r, _ = b.result(0)
            b.release()
            return r

        def via_split():
            return split.compact_split(eng, job, [(0, 0), (len(js.a), n - len(js.a))], split.SingleRank(), 0)

        r = direct()
        s = via_split()
        same = np.array_equal(out.download(r.block_count * bs), s.blocks.download(r.block_count * bs))
        td, tsp = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            direct()
            td.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            s = via_split()
            tsp.append(time.perf_counter() - t0)
            s.blocks.free()
        md, ms = sorted(td)[len(td) // 2], sorted(tsp)[len(tsp) // 2]
        print(json.dumps({"probe": "split_single_rank", "values": n, "blocks": int(r.block_count),
                          "identical_blocks": bool(same), "direct_ms": round(md * 1e3, 3),
                          "split_ms": round(ms * 1e3, 3), "overhead": round(ms / md, 3)}))


if __name__ == "__main__":
    main()
