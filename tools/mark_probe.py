"""Cost of the per-kernel timing marks (TBC_CONFIG_PROFILE hipEvents between
a batch's kernels): the same bench workload timed with the engine's profile
flag on and off, interleaved.

  python tools/mark_probe.py --config 3 --steps 10 --reps 3
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tigerbeetle_amd import Engine, configs  # noqa: E402
from tigerbeetle_amd.shard import plan_shards  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    bs = 1 << 20
    njobs = configs.DEFAULT_JOBS.get(args.config, 1)
    res = {"on": [], "off": []}
    for rep in range(args.reps):
        for prof in (True, False):
            with Engine(device=0, block_size=bs, profile=prof, arena_bytes=2 << 30) as eng:
                plan = plan_shards([configs.job_bytes(args.config, j) for j in range(njobs)], 1)
                wl = bench.Workload(eng, args.config, plan[0], bs)
                for _ in range(3):
                    wl.step(eng).release()
                eng.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    wl.step(eng).release()
                eng.synchronize()
                res["on" if prof else "off"].append(round((time.perf_counter() - t0) / args.steps * 1e3, 3))
                del wl
    print(json.dumps({"config": args.config, "ms_per_step": res}))


if __name__ == "__main__":
    main()
