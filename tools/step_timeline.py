"""One bench step's device timeline from a rocprofv3 kernel trace: the last
step (the bench runs one more after the timed ones) split out by the first
kernel of a step, every kernel with its queue, start offset and duration,
and the gaps on the engine queue.

  python tools/step_timeline.py <dir>/run_kernel_trace.csv FIRST_KERNEL [--all]
"""
import csv
import sys

path, first = sys.argv[1], sys.argv[2]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
i0, i1 = starts[-2], starts[-1]  # the step before the last one (the last may trail)
step = rows[i0:i1]
t0 = int(step[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in step)
busy, last_end = 0, t0
for r in step:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tbc::", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "--all" in sys.argv:
        print(f"q{r['Queue_Id']} +{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f} us  {name[:60]}")
    if r["Queue_Id"] == step[0]["Queue_Id"]:
        busy += e - max(s, last_end) if e > last_end else 0
        last_end = max(last_end, e)
print(f"step span {(end - t0) / 1e3:.1f} us, engine queue busy {busy / 1e3:.1f} us, kernels {len(step)}")
