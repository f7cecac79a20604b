"""One bench step's kernel/copy timeline from a scripts/trace_steps.sh run, as CSV.

usage: python scripts/timeline_summary.py <trace dir> <out.csv>
Takes the second-to-last scan/dense kernel launch as the step anchor and lists every
kernel and copy from the end of the previous step's readback to the next step's first
operation: start (us, relative), duration (us), gap since the previous operation (us).
"""
import csv
import sys

src, dst = sys.argv[1], sys.argv[2]
ev = []
for r in csv.DictReader(open(f"{src}/run_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60]))
try:
    for r in csv.DictReader(open(f"{src}/run_memory_copy_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
except FileNotFoundError:
    pass
ev.sort()
anchors = [i for i, e in enumerate(ev) if "scan_kernel" in e[2] or "dense_kernel" in e[2]]
a, b = anchors[-3], anchors[-2]
i0 = a
while i0 > 0 and "copy" not in ev[i0][2]:
    i0 -= 1
rows = ev[i0:b]
t0 = rows[0][0]
with open(dst, "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["op", "start_us", "dur_us", "gap_us"])
    prev_end = rows[0][0]
    for s, e, name in rows:
        w.writerow([name, round((s - t0) / 1e3, 1), round((e - s) / 1e3, 1), round((s - prev_end) / 1e3, 1)])
        prev_end = max(prev_end, e)
    w.writerow(["next step", round((ev[b][0] - t0) / 1e3, 1), "", ""])
print(open(dst).read())
