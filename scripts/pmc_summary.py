"""Summarise rocprofv3 counter CSVs: mean per dispatch of each counter for one kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "scan_kernel"
for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[-2], {k: f"{sum(v) / len(v):.4g}" for k, v in agg.items()})
for f in glob.glob(f"{root}/trace/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if pat in r["Name"]:
            print("trace", r["Name"][:60], "calls", r["Calls"], "avg_ns", r["AverageNs"])
