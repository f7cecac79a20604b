"""One bench step's kernel/copy timeline from a scripts/trace_steps.sh run, as CSV.

usage: python scripts/timeline_summary.py <trace dir> <out.csv> [step]
trace_steps.sh runs one warm-up and five timed steps, then the untimed stage-timing step
(and, for --shard-of, the whole-genome parity search).  The anchor is the scan (or dense)
kernel of timed step `step` (default 3, 1-based among the timed steps); rows run from the
previous step's last operation to the next step's scan kernel: start (us, relative to the
first row), duration (us), gap since the previous operation ended (us).
"""
import csv
import sys

src, dst = sys.argv[1], sys.argv[2]
step = int(sys.argv[3]) if len(sys.argv) > 3 else 3
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
a, b = anchors[step], anchors[step + 1]  # anchors[0] is the warm-up step
rows = ev[a - 1:b]
t0 = rows[0][0]
with open(dst, "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["op", "start_us", "dur_us", "gap_us"])
    prev_end = rows[0][0]
    for s, e, name in rows:
        w.writerow([name, round((s - t0) / 1e3, 1), round((e - s) / 1e3, 1), round((s - prev_end) / 1e3, 1)])
        prev_end = max(prev_end, e)
    w.writerow(["next step", round((ev[b][0] - t0) / 1e3, 1), "", ""])
    w.writerow(["step (scan start to next scan start)", round((ev[b][0] - ev[a][0]) / 1e3, 1), "", ""])
print(open(dst).read())
