"""A/B of the hit-order modes on one resident c3 workload: stage times per mode.
usage: python scripts/ab_order.py [--scale S] [--shard-of N] [--config c3]"""
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
ap.add_argument("--scale", type=float, default=1.0)
ap.add_argument("--shard-of", type=int, default=0)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
cfg = synth.CONFIGS[args.config]
total = int(cfg["total"] * args.scale) // 64 * 64
sts = synth.make_sts(cfg["n_sts"], W=cfg["W"], iupac=cfg["iupac"])
eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
with tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False) as fh:
    fh.write(sts.text())
eng.load_sts_file(fh.name)
table = eng.device_table()
dev = torch.device("cuda", 0)
names, lens, buf, offs, planted = synth.build_genome_torch(total, cfg["records"], sts, seed=1, N=cfg["N"], M=cfg["M"],
                                                          W=cfg["W"], nrun=cfg["nrun"], device=dev)
stream = torch.cuda.current_stream().cuda_stream
g = _native.Genome(0, lens)
for r, n in enumerate(lens):
    g.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
g.seal(stream)
rng = shard_ranges(lens, args.shard_of)[0] if args.shard_of > 1 else None
ref = None
for mode in ("radix64", "scatter", "auto"):
    s = _native.Search(table, g)
    s.set_options(sort=mode)
    s.set_stage_timing(True)
    rows = []
    for _ in range(args.reps + 2):
        n = s.run(rng, stream)
        rows.append(s.last_stats())
    hits = s.fetch(n)
    if ref is None:
        ref = hits
    same = hits.tobytes() == ref.tobytes()
    st = rows[2:]
    print(f"{mode:8s} hits={n} same={same} " + " ".join(
        f"{k}={np.mean([r[k] for r in st]):.4f}" for k in ("scan_ms", "tail_ms", "pair_ms", "order_ms")), flush=True)
    s.set_stage_timing(False)
    s.set_scan_timing(False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        s.run(rng, stream)
    torch.cuda.synchronize()
    print(f"{mode:8s} untimed run {1e3 * (time.perf_counter() - t) / 20:.4f} ms", flush=True)
    s.close()
