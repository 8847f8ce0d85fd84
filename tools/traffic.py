"""Summarise a tools/profile.sh run into profiles/<tag>/.

    python tools/traffic.py gpurun_out/prof_<tag> profiles/<tag>

Writes kernel_stats.csv (rocprofv3 --stats), bench.json, and traffic.json:
per kernel, the average launch duration from the kernel trace and the HBM
bytes per launch from the PMC passes, corrected as MI355X_MICROARCH.md
§HBM prescribes (FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
tallies 128-byte requests at 64 bytes, so it is doubled). bench.py reports
`roofline.traffic` from traffic.json only when its lib_md5 matches the
libtbc.so being benchmarked.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import shutil
import sys


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").split("<")[0]  # template arguments may hold "::"
    return n.split("::")[-1]


def find(root: str, pattern: str) -> str:
    hits = glob.glob(os.path.join(root, "**", pattern), recursive=True)
    if not hits:
        raise SystemExit(f"no {pattern} under {root}")
    return hits[0]


def inst(name: str) -> str:
    """The instantiation: the short name with its template arguments."""
    return name.split("(")[0].replace("void ", "").replace("tbc::", "").strip()


def counters(root: str, counter: str) -> dict:
    per = collections.defaultdict(list)
    for row in csv.DictReader(open(find(root, "*counter_collection.csv"))):
        if row["Counter_Name"] == counter:
            per[inst(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


SQ_COUNTERS = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES",
               "SQ_INSTS_SALU", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"]


def main() -> None:
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    stats = find(os.path.join(src, "trace"), "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
    # Every instantiation has its own entry (e.g. the fused and the chain-only
    # k_data_blocks); the short name carries the heaviest instantiation's
    # numbers, durations and counters alike (bench.py looks kernels up by it).
    avg_ns, tot_ns, calls, heaviest = {}, {}, {}, {}
    for r in csv.DictReader(open(stats)):
        i, k = inst(r["Name"]), short(r["Name"])
        avg_ns[i], tot_ns[i], calls[i] = float(r["AverageNs"]), float(r["TotalDurationNs"]), int(r["Calls"])
        if k not in heaviest or tot_ns[i] > tot_ns[heaviest[k]]:
            heaviest[k] = i
    fetch = counters(os.path.join(src, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(src, "write"), "WRITE_SIZE")
    md5 = open(os.path.join(src, "lib.md5")).read().split()[0]
    bench_cfg = None
    try:
        bench_cfg = json.loads(open(os.path.join(src, "bench.json")).read())["config"].get("baseline_config")
    except (OSError, ValueError, KeyError):
        pass
    sq = {}
    if glob.glob(os.path.join(src, "sq", "**", "*counter_collection.csv"), recursive=True):
        for c in SQ_COUNTERS:
            for k, v in counters(os.path.join(src, "sq"), c).items():
                sq.setdefault(k, {})[c] = v
    out = {"lib_md5": md5, "baseline_config": bench_cfg, "note": "bytes per launch; fetch = 2 x FETCH_SIZE KiB (gfx950 correction), "
                                   "write = WRITE_SIZE KiB", "kernels": {}}
    names = sorted(set(avg_ns) | set(heaviest))
    for k in names:
        i = heaviest.get(k, k)  # a short name: its heaviest instantiation
        f = fetch.get(i, 0.0) * 1024 * 2
        w = write.get(i, 0.0) * 1024
        out["kernels"][k] = {"avg_ns": avg_ns[i], "calls": calls[i], "fetch_bytes": round(f), "write_bytes": round(w),
                             "traffic_bytes": round(f + w),
                             "traffic_gbs": round((f + w) / avg_ns[i], 1) if avg_ns[i] else None}
        if k != i:
            out["kernels"][k]["instantiation"] = i
        if i in sq:
            s = dict(sq[i])
            # Rates against the chip: a wave64 VALU instruction holds a SIMD-32 for 2 cycles
            # (1,024 SIMDs); LDS instructions per CU-cycle (256 CUs). Busy cycles are per-SE
            # sums (SQ counters count quad-cycles for WAVE/WAIT/ACTIVE: MI355X_MICROARCH.md).
            ns = avg_ns[i]
            if ns:
                s["valu_instr_per_ns"] = round(s.get("SQ_INSTS_VALU", 0) / ns, 2)
                s["valu_issue_frac"] = round(s.get("SQ_INSTS_VALU", 0) * 2 / (1024 * 2.4 * ns), 4)
                s["lds_instr_per_ns"] = round(s.get("SQ_INSTS_LDS", 0) / ns, 2)
                s["lds_instr_frac"] = round(s.get("SQ_INSTS_LDS", 0) * 2 / (256 * 2.4 * ns), 4)
            out["kernels"][k]["sq"] = s
    json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
