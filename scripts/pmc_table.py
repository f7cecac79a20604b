"""Mean per-dispatch counter values of rocprofv3 CSV output directories."""
import collections
import csv
import glob
import os
import sys


def summarize(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    agg = collections.defaultdict(float)
    disp = set()
    for r in rows:
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    per = collections.defaultdict(list)
    for (dd, c), v in agg.items():
        per[c].append(v)
    return {c: sum(v) / len(v) for c, v in per.items()}


if __name__ == "__main__":
    for d in sorted(glob.glob(os.path.join(sys.argv[1], "*"))):
        if os.path.isdir(d) and os.path.exists(os.path.join(d, "run_counter_collection.csv")):
            s = summarize(d)
            print(os.path.basename(d), " ".join(f"{k}={v:.4g}" for k, v in sorted(s.items())))
