"""Config 1 engine-queue gap attribution from a rocprofv3 kernel trace:
passes are split at idle periods > 2 ms (whole chip idle); in the last pass
every gap on the engine queue (the queue of k_grid_resolve) is attributed to
what ended just before the next engine kernel started: a tail kernel (the
engine waited for a tail's event), or nothing (host enqueue lag).

  python tools/c1_gaps.py <trace.csv> [--list N]
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tbc::", "")[:40]
S = lambda r: int(r["Start_Timestamp"])
E = lambda r: int(r["End_Timestamp"])
eng = collections.Counter(r["Queue_Id"] for r in rows if "k_grid_resolve" in r["Kernel_Name"]).most_common(1)[0][0]
passes, cur, end = [], [], 0
for r in rows:
    if cur and S(r) - end > 2_000_000:
        passes.append(cur)
        cur = []
    cur.append(r)
    end = max(end, E(r))
passes.append(cur)
print("passes:", [(len(p), round((max(E(r) for r in p) - S(p[0])) / 1e6, 2)) for p in passes])
p = passes[-1]
t0 = S(p[0])
span = max(E(r) for r in p) - t0
er = [r for r in p if r["Queue_Id"] == eng]
busy = 0
last = S(er[0])
for r in er:
    busy += max(0, E(r) - max(S(r), last))
    last = max(last, E(r))
gaps = []
for a, b in zip(er, er[1:]):
    g = S(b) - E(a)
    if g <= 0:
        continue
    # the latest non-engine kernel ending inside (E(a), S(b)]
    cause = None
    for r in p:
        if r["Queue_Id"] != eng and E(a) < E(r) <= S(b):
            if cause is None or E(r) > E(cause):
                cause = r
    gaps.append((g, name(a), name(b), (name(cause), S(b) - E(cause)) if cause else None))
tot = sum(g for g, *_ in gaps)
by_pair = collections.defaultdict(lambda: [0, 0])
for g, a, b, c in gaps:
    k = (a, b, "tail" if c and c[1] < 20_000 else "host")
    by_pair[k][0] += g
    by_pair[k][1] += 1
print(f"last pass: span {span / 1e6:.2f} ms, engine busy {busy / 1e6:.2f} ms, gaps {tot / 1e6:.2f} ms in {len(gaps)}, kernels {len(p)} ({len(er)} engine)")
for k, (g, n) in sorted(by_pair.items(), key=lambda x: -x[1][0])[:25]:
    print(f"{g / 1e6:7.3f} ms {n:5d}  {k[0]:>32} -> {k[1]:<32} {k[2]}")
tail_wait = sum(g for g, a, b, c in gaps if c and c[1] < 20_000)
print(f"gaps ending <20us after a tail kernel: {tail_wait / 1e6:.2f} ms")
ek = collections.defaultdict(lambda: [0, 0])
for r in er:
    ek[name(r)][0] += E(r) - S(r)
    ek[name(r)][1] += 1
print("engine kernels:")
for k, (t, n) in sorted(ek.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{t / 1e6:7.3f} ms {n:5d}  {k}")
