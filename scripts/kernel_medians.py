"""Median duration of each kernel in a rocprofv3 kernel trace (us), and the median gap from one
kernel's end to the next kernel's start on the same queue.  usage: kernel_medians.py <trace csv>"""
import collections
import csv
import statistics
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48],
               r.get("Queue_Id", "?")) for r in csv.DictReader(open(sys.argv[1])))
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
last = {}
for s, e, n, q in rows:
    dur[n].append((e - s) / 1e3)
    if q in last:
        gap[(last[q][1], n)].append((s - last[q][0]) / 1e3)
    last[q] = (e, n)
for n, v in sorted(dur.items(), key=lambda x: -statistics.median(x[1]) * len(x[1])):
    if "mp::" in n:
        print(f"{n:50s} n={len(v):4d} median {statistics.median(v):8.1f} us  min {min(v):8.1f}")
for (a, b), v in sorted(gap.items()):
    if "mp::" in a and "mp::" in b and len(v) > 5:
        print(f"gap {a[:30]:30s} -> {b[:30]:30s} median {statistics.median(v):6.1f} us")
