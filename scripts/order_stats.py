"""Hit-order bucket statistics of one resident workload (the order stage's shape):
how the hits spread over the device sort's buckets (equal ranges of global position, as
sort_plan cuts them), and how many buckets exceed the wave (64), workgroup (256) and crowded
(2,048) limits.  usage: python scripts/order_stats.py [--config c4]"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
args = ap.parse_args()
import torch  # noqa: E402
from merpcr_amd import MerPCR, _native, synth  # noqa: E402

cfg = synth.CONFIGS[args.config]
sts = synth.make_sts(cfg["n_sts"], W=cfg["W"], iupac=cfg["iupac"])
eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
with tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False) as fh:
    fh.write(sts.text())
eng.load_sts_file(fh.name)
table = eng.device_table()
names, lens, buf, offs, _ = synth.build_genome_torch(cfg["total"], cfg["records"], sts, seed=1, N=cfg["N"], M=cfg["M"],
                                                     W=cfg["W"], nrun=cfg["nrun"], device=torch.device("cuda", 0))
g = _native.Genome(0, lens)
for r, n in enumerate(lens):
    g.put_device(r, buf.data_ptr() + int(offs[r]), n)
g.seal()
s = _native.Search(table, g)
n = s.run()
hits = s.fetch(n)
base = np.zeros(len(lens) + 1, dtype=np.int64)
base[1:] = np.cumsum([(x + 63) // 64 * 64 for x in lens])
gk = base[hits["seq"].astype(np.int64)] + hits["pos1"].astype(np.int64)
total = int(base[-1])
for nb in (1 << 14, 1 << 15, 1 << 16, 1 << 17):
    span = -(-total // nb)
    c = np.bincount(gk // span, minlength=nb)
    print(f"buckets {nb}: mean {c.mean():.1f} max {c.max()}  >64: {(c > 64).sum()} (hits {c[c > 64].sum()})  "
          f">256: {(c > 256).sum()} (hits {c[c > 256].sum()})  >2048: {(c > 2048).sum()}")
u, cnt = np.unique(gk, return_counts=True)
print(f"hits {n}, distinct positions {len(u)}, positions with > 64 hits: {(cnt > 64).sum()} (hits {cnt[cnt > 64].sum()}), "
      f"max per position {cnt.max()}")
hist = np.histogram(cnt, bins=[1, 2, 3, 5, 9, 17, 33, 65, 129, 257, 513, 1025, 2049, 1 << 30])
print("hits per position:", [(int(a), int(b)) for a, b in zip(hist[1], hist[0])])
