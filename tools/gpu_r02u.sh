#!/bin/bash
# Per-launch kernel trace of config 3 (sort passes in order).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02u
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last step: from the last k_sort_extract onwards
idx = [i for i, r in enumerate(rows) if "k_sort_extract" in r["Kernel_Name"]]
for r in rows[idx[-1]: idx[-1] + 40]:
    print(r["Kernel_Name"].split("(")[0][-40:], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0, r.get("Grid_Size", ""))
PY
