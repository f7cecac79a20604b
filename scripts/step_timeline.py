"""Per-step kernel timeline of a traced bench run (rocprofv3 --kernel-trace csv): for each scan
launch, its duration, the gap to the previous kernel on the GPU, and the kernels between it and
the next scan (with their overlap).  usage: python scripts/step_timeline.py <run_kernel_trace.csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:40],
       r.get("Queue_Id", "")) for r in rows]
scans = [i for i, e in enumerate(ev) if "scan_kernel" in e[2]]
steps = []
for a, b in zip(scans, scans[1:]):
    t0 = ev[a][0]
    steps.append((ev[b][0] - t0) / 1000)
print(f"scan launches {len(scans)}; scan-start to scan-start (us): "
      f"median {sorted(steps)[len(steps) // 2]:.1f} min {min(steps):.1f}" if steps else "fewer than 2 scans")
for a, b in list(zip(scans, scans[1:]))[-n_show:]:
    t0 = ev[a][0]
    print("---")
    for e in ev[a:b + 1]:
        print(f"  {(e[0] - t0) / 1000:8.1f} .. {(e[1] - t0) / 1000:8.1f}  ({(e[1] - e[0]) / 1000:7.1f})  q{e[3]:>3} {e[2]}")
