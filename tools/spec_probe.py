"""Timing probe of the speculated producers (TBC_COMPACTION_UNIQUE_KEYS), no chains.

Runs a few BASELINE config-2 (or -4) jobs with TBC_PROBE_PRODUCERS_ONLY=1:
the fused block kernel runs its producers only, and each speculated
producer writes its wall-clock split (100 MHz ticks: waiting for windows,
searching, histogram, rest, steps) into its block's header bytes. Prints
per-step averages in microseconds. Output blocks are not valid in this mode.

  TBC_PROBE_PRODUCERS_ONLY=1 python tools/spec_probe.py --config 2 --jobs 4
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tigerbeetle_amd import Engine, Job, abi, configs  # noqa: E402
from tigerbeetle_amd.engine import stage_blocks  # noqa: E402
from tigerbeetle_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--first", type=int, default=0)
    args = ap.parse_args()
    assert os.environ.get("TBC_PROBE_PRODUCERS_ONLY"), "set TBC_PROBE_PRODUCERS_ONLY=1"
    bs = 1 << 20
    with Engine(device=0, block_size=bs, profile=True) as eng:
        jobs, keep = [], []
        base = 1
        for g in range(args.first, args.first + args.jobs):
            js = configs.GENERATORS[args.config](g)
            if not js.unique_keys:
                continue
            lay = js.tree.layout(bs)
            vcm = lay["block_value_count_max"]
            if js.a_immutable:
                abuf = eng.upload(js.a)
                if js.a_unsorted:
                    eng.sort_values(js.tree, abuf, len(js.a))
                segs_a = [(abuf.ptr, len(js.a))]
                keep.append(abuf)
            else:
                ab, segs_a = stage_blocks(eng, [workloads.split_blocks(js.a, vcm)], js.tree.value_size, bs)
                keep.append(ab)
            bb, segs_b = stage_blocks(eng, [workloads.split_blocks(t, vcm) for t in js.b_tables], js.tree.value_size, bs)
            keep.append(bb)
            reservation = (len(js.b_tables) + 1) * lay["block_count_max"]
            out = eng.alloc(reservation * bs)
            keep.append(out)
            addrs = np.arange(base, base + reservation, dtype=np.uint64)
            base += reservation
            jobs.append(Job(js.tree, segs_a, segs_b, js.a_immutable, js.drop_tombstones, js.level_b, 1, 48, addrs,
                            out, flags=abi.COMPACTION_UNIQUE_KEYS))
        for rep in range(2):
            b = eng.submit(jobs)
            b.wait()
            times = b.kernel_times()
            blocks = []
            for i, job in enumerate(jobs):
                r, _ = b.result(i)
                img = job.output.download(r.block_count * bs).reshape(-1, bs)
                for s in range(r.block_count):
                    if img[s, 240] == 4:  # index block (written by k_index_blocks)
                        continue
                    blocks.append(img[s, :40].view(np.uint64).copy())
            b.release()
        t = np.array(blocks, dtype=np.float64)
        t = t[t[:, 4] > 0]
        per_step = t[:, :4].sum(axis=0) / t[:, 4].sum() / 100.0  # 100 MHz ticks -> us
        total = t[:, :4].sum(axis=1) / 100.0
        print(json.dumps({"config": args.config, "blocks": int(len(t)), "steps_per_block": float(t[:, 4].mean()),
                          "us_per_step": {"wait": round(per_step[0], 3), "search": round(per_step[1], 3),
                                          "hist": round(per_step[2], 3), "rest": round(per_step[3], 3)},
                          "block_us": {"mean": round(float(total.mean()), 1), "max": round(float(total.max()), 1)},
                          "kernel_us": {k: round(v, 1) for k, v in times.items()}}))


if __name__ == "__main__":
    main()
