"""Per-wave timeline of scan_kernel (ablation variant 40: wall-clock stamps at entry, after the
LDS staging, at the end of the super-step loop and at exit), for one resident c3 workload.
usage: python scripts/wave_times.py [--shard-of N] [--config c3]
Prints, in microseconds from the first wave's entry: the spread of entries, staging ends,
loop ends and exits (min / median / p90 / max) and the mean loop time per wave."""
import argparse
import ctypes
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--shard-of", type=int, default=8)
ap.add_argument("--build-only", action="store_true")
ap.add_argument("--no-build", action="store_true", help="use the variant library built beforehand (CPU side)")
args = ap.parse_args()
from merpcr_amd import _build  # noqa: E402
import ablate_variants  # noqa: E402
VAR = int(os.environ.get("MP_WAVE_VARIANT", "40"))
path = os.path.join(_build.LIBDIR, f"libmerpcr_hip_ablate{VAR}.so")
if not (args.no_build and os.path.exists(path)):
    src = ablate_variants.make_source_dir(VAR, _build.CSRC, os.path.join(tempfile.gettempdir(), f"mp_ablate_{VAR}"))
    _build.build_native(lib=path, src_dir=src, tag=f"_ablate{VAR}")
if args.build_only:
    sys.exit(0)
import torch  # noqa: E402
from merpcr_amd import MerPCR, _native, synth  # noqa: E402
from merpcr_amd.dist import shard_ranges  # noqa: E402
lib = ctypes.CDLL(path)
_native._sig(lib)
_native._lib = lib
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
rng = shard_ranges(lens, args.shard_of)[0] if args.shard_of > 1 else None
for _ in range(3):
    s.run(rng)
print("scan_ms", s.last_stats()["scan_ms"])
out = (ctypes.c_uint64 * (8192 * 4))()
lib.mp_debug_wave_times.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
assert lib.mp_debug_wave_times(ctypes.cast(out, ctypes.c_void_p), 8192) == 0
t = np.frombuffer(out, dtype=np.uint64).reshape(8192, 4).astype(np.int64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
us = (t - t0) / 100.0  # wall_clock64: 100 MHz
ids = np.nonzero(np.frombuffer(out, dtype=np.uint64).reshape(8192, 4)[:, 0] > 0)[0]
nss = t[:, 3].copy()
t[:, 3] = t[:, 2]
us = (t - t0) / 100.0
blk, wv = ids // 16, ids % 16
print("super-steps per wave: mean %.1f min %d max %d" % (nss.mean(), nss.min(), nss.max()))
for grp in range(8):
    m = blk % 8 == grp
    print(f"XCD group {grp}: loop end mean {us[m, 2].mean():8.1f} max {us[m, 2].max():8.1f}  super-steps mean "
          f"{nss[m].mean():.1f} (us per super-step {np.mean((us[m, 2] - us[m, 1]) / np.maximum(nss[m], 1)):.2f})")
print("by wave slot w: loop end mean", [round(float(us[wv == k, 2].mean()), 1) for k in range(16)])
print("by wave slot w: super-steps mean", [round(float(nss[wv == k].mean()), 1) for k in range(16)])
for i, name in enumerate(("entry", "staged", "loop end")):
    c = us[:, i]
    print(f"{name:9s} min {c.min():8.1f} med {np.median(c):8.1f} p90 {np.percentile(c, 90):8.1f} max {c.max():8.1f}")
loop = us[:, 2] - us[:, 1]
print(f"loop per wave: mean {loop.mean():.1f} min {loop.min():.1f} max {loop.max():.1f} us; waves {len(t)}")
hist = np.histogram(us[:, 2], bins=12)
print("loop-end histogram:", [(round(float(e), 1), int(c)) for e, c in zip(hist[1], hist[0])])
if hasattr(lib, "mp_debug_ss_times"):  # variant 42: each wave's first 32 super-step ends
    ss = (ctypes.c_uint64 * (8192 * 32))()
    lib.mp_debug_ss_times.argtypes = [ctypes.c_void_p]
    assert lib.mp_debug_ss_times(ctypes.cast(ss, ctypes.c_void_p)) == 0
    a = np.frombuffer(ss, dtype=np.uint64).reshape(8192, 32).astype(np.int64)[ids]
    st = (np.frombuffer(out, dtype=np.uint64).reshape(8192, 4).astype(np.int64)[ids, 1])[:, None]
    prev = np.concatenate([st, a[:, :-1]], axis=1)
    dur = (a - prev) / 100.0
    ok = a > 0
    print("super-step k of a wave (us): mean duration by k, waves reaching it")
    print([(k, round(float(dur[ok[:, k], k].mean()), 2), int(ok[:, k].sum())) for k in range(32) if ok[:, k].any()])
    fin = (a[:, 0] - t0) / 100.0
    print(f"first super-step end: min {fin.min():.1f} med {np.median(fin):.1f} max {fin.max():.1f} us")
