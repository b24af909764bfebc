"""Kernel timeline of non-rebuild steps in a rocprofv3 kernel trace of bench.py: the
dispatches between consecutive k_final_initial launches that contain no neighbour build,
with the gap before each, and per step the kernel time, the gap time and the wall span.
usage: python tools/step_timeline.py trace.csv [steps_to_print=1]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
show = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
marks = [k for k, n in enumerate(names) if "k_final_initial" in n]
steps = []
for a, b in zip(marks, marks[1:]):
    seg = rows[a:b]
    if any("k_blk_build" in r["Kernel_Name"] or "k_blk_neigh" in r["Kernel_Name"] for r in seg):
        continue
    steps.append(seg)
if not steps:
    sys.exit("no non-rebuild step in the trace")
spans, kts, gaps = [], [], []
for seg in steps:
    t0 = int(seg[0]["Start_Timestamp"])
    prev = t0
    kt = gp = 0.0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gp += max(s - prev, 0) / 1e3
        kt += (e - s) / 1e3
        prev = max(prev, e)
    spans.append((prev - t0) / 1e3)
    kts.append(kt)
    gaps.append(gp)
for seg in steps[-show:]:
    t0 = int(seg[0]["Start_Timestamp"])
    prev = t0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%8.1f gap %6.1f dur %7.1f  %s" % ((s - t0) / 1e3, max(s - prev, 0) / 1e3,
                                                (e - s) / 1e3, r["Kernel_Name"][:90]))
        prev = max(prev, e)
    print("--")
n = len(steps)
print("non-rebuild steps %d: span %.1f us, kernels %.1f us, gaps %.1f us (means); launches/step %.1f"
      % (n, sum(spans) / n, sum(kts) / n, sum(gaps) / n, sum(len(s) for s in steps) / n))
