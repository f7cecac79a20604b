"""Per-kernel-form summary of rocprofv3 output directories: trace durations (median of each
form's dispatches) and PMC counters (mean per dispatch, instances summed), one line per form.
usage: python scripts/pmc_forms.py <dir> [<dir> ...] [--match scan_kernel] [--json out.json]
A <dir> holds rocprofv3 -d output (any depth): *kernel_trace.csv and/or *counter_collection.csv."""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def short(name: str) -> str:
    return name.replace("void mp::", "").replace("(mp::ScanArgs)", "")


def summarize(d: str, match: str) -> dict:
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in dur.items():
            out[k]["calls"] = len(v)
            out[k]["median_us"] = round(statistics.median(v) / 1e3, 2)
            out[k]["min_us"] = round(min(v) / 1e3, 2)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        agg = collections.defaultdict(list)
        for (dsp, c), v in per.items():
            agg[(names[dsp], c)].append(v)
        for (k, c), v in agg.items():
            out[k][c] = sum(v) / len(v)
    return dict(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="_kernel")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    res = {}
    for d in a.dirs:
        res[d] = summarize(d, a.match)
        for k, v in sorted(res[d].items()):
            cs = " ".join(f"{c}={x:.4g}" for c, x in sorted(v.items()) if c not in ("calls", "median_us", "min_us"))
            print(f"{os.path.basename(d.rstrip('/')):14s} {k[:60]:60s} calls={v.get('calls', '-')} "
                  f"med={v.get('median_us', '-')}us {cs}")
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
