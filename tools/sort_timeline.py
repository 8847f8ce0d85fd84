"""The last memtable sort's kernel timeline from a rocprofv3 kernel trace.

  python tools/sort_timeline.py gpurun_out/<dir>/trace_c3/run_kernel_trace.csv
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
i0 = [i for i, r in enumerate(rows) if "k_sort_extract" in r["Kernel_Name"]][-1]
seq = []
for r in rows[i0:]:
    name = r["Kernel_Name"].split("(")[0].replace("tbc::", "")
    seq.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Start_Timestamp"])))
    if "k_sort_rescue" in name:
        break
t0 = seq[0][2]
for name, d, s in seq:
    print(f"{name:20s} {d:8.1f} us  start +{(s - t0) / 1e3:8.1f}")
print(f"span {(seq[-1][2] - t0) / 1e3 + seq[-1][1]:.1f} us")
