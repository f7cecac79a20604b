"""Kernel intervals of a few consecutive bench steps from a trace_steps.sh run (several
streams: intervals may overlap).  usage: python scripts/timeline_streams.py <trace dir> [first] [count]
Prints each kernel of timed steps first..first+count-1 (1-based, by scan launch order) with its
queue, start and end (us, relative to the first printed scan's start), and the average
scan-start-to-scan-start interval of the timed steps."""
import csv
import sys

src = sys.argv[1]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 2
count = int(sys.argv[3]) if len(sys.argv) > 3 else 2
ev = []
for r in csv.DictReader(open(f"{src}/run_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:50],
               r.get("Queue_Id", r.get("Stream_Id", "?"))))
ev.sort()
scans = [i for i, e in enumerate(ev) if "scan_kernel" in e[2] or "dense_kernel" in e[2]]
a, b = scans[first], scans[min(first + count, len(scans) - 1)]
t0 = ev[a][0]
for s, e, name, q in ev[a:b + 1]:
    print(f"{name:52s} q={q:>3} start={(s - t0) / 1e3:9.1f} end={(e - t0) / 1e3:9.1f} dur={(e - s) / 1e3:8.1f}")
timed = scans[1:6]
d = [(ev[timed[i + 1]][0] - ev[timed[i]][0]) / 1e3 for i in range(len(timed) - 1)]
print("scan-to-scan intervals (timed steps):", [round(x, 1) for x in d])
