"""Scan-kernel and whole-run time against shard size (rank 0's range of an N-way split) on
one resident c3 workload: the fixed per-run cost is the intercept.
usage: python scripts/shard_curve.py [--config c3] [--parts 1,2,4,8,16,32,64,128]"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from merpcr_amd import MerPCR, _native, synth  # noqa: E402
from merpcr_amd.dist import shard_ranges  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--parts", default="1,2,4,8,16,32,64,128")
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
cfg = synth.CONFIGS[args.config]
sts = synth.make_sts(cfg["n_sts"], W=cfg["W"], iupac=cfg["iupac"])
eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
with tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False) as fh:
    fh.write(sts.text())
eng.load_sts_file(fh.name)
table = eng.device_table()
names, lens, buf, offs, planted = synth.build_genome_torch(cfg["total"], cfg["records"], sts, seed=1, N=cfg["N"],
                                                          M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"],
                                                          device=torch.device("cuda", 0))
stream = torch.cuda.current_stream().cuda_stream
g = _native.Genome(0, lens)
for r, n in enumerate(lens):
    g.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
g.seal(stream)
s = _native.Search(table, g)
rows = []
for parts in [int(x) for x in args.parts.split(",")]:
    rng = shard_ranges(lens, parts)[0] if parts > 1 else None
    s.set_stage_timing(True)
    st = []
    for _ in range(args.reps + 2):
        s.run(rng, stream)
        st.append(s.last_stats())
    st = st[2:]
    s.set_stage_timing(False)
    s.set_scan_timing(False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.reps):
        s.run(rng, stream)
    torch.cuda.synchronize()
    run_ms = (time.perf_counter() - t) / args.reps * 1e3
    s.set_scan_timing(True)
    m = {k: float(np.mean([r[k] for r in st])) for k in ("scan_ms", "tail_ms", "pair_ms", "order_ms")}
    rows.append((1.0 / parts, m["scan_ms"], run_ms))
    print(f"1/{parts:<4d} scan {m['scan_ms']:.4f} tail {m['tail_ms']:.4f} pair {m['pair_ms']:.4f} "
          f"order {m['order_ms']:.4f} | untimed run {run_ms:.4f} ms", flush=True)
x = np.array([r[0] for r in rows])
for j, name in ((1, "scan"), (2, "run")):
    y = np.array([r[j] for r in rows])
    b, a = np.polyfit(x, y, 1)
    print(f"{name}: {a * 1e3:.1f} us fixed + {b:.4f} ms per whole genome")
