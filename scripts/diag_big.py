"""Diagnostic: the 4.5 Gbp test genome (tests/test_gpu_fullscale.py::test_genome_past_2_32),
GPU vs C oracle, with the missing / extra hits binned by record and position, and the hit
count under several kernel-path options."""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from merpcr_amd import MerPCR, _native, synth  # noqa: E402
from oracle import c_oracle as C  # noqa: E402
from oracle import epcr_oracle as O  # noqa: E402

lens = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2300000000,1200000000,1000000000").split(",")]
cfg = synth.CONFIGS["c3"]
total = sum(lens)
sts = synth.make_sts(cfg["n_sts"], W=cfg["W"])
eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
with tempfile.TemporaryDirectory() as td:
    p = os.path.join(td, "c.sts")
    open(p, "w").write(sts.text())
    assert eng.load_sts_file(p)
table = eng.device_table()
dev = torch.device("cuda", 0)
names, lens, buf, offs, planted = synth.build_genome_torch(
    total, len(lens), sts, seed=3, N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=dev, lens=lens)
synth.plant_at_ends(buf, offs, lens, sts)
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
genome = _native.Genome(0, lens)
for r, n in enumerate(lens):
    genome.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
genome.seal(stream)
res = {}
for name, opts in [("default", {}), ("sort_rocprim", dict(sort="rocprim")), ("tails_inline", dict(tails="inline")),
                   ("no_defer", dict(defer=False))]:
    s = _native.Search(table, genome)
    try:
        if opts:
            s.set_options(**opts)
        got = s.fetch(s.run(None, stream))
        res[name] = got
        print(name, len(got), s.last_stats(), flush=True)
    except Exception as e:  # noqa: BLE001
        print(name, "error", e, flush=True)
    s.close()
genome.close()
host = buf.cpu().numpy()
del buf
seqs = [host[int(offs[r]):int(offs[r]) + lens[r]] for r in range(len(lens))]
otable = O.load_sts_lines(sts.text().splitlines(True), cfg["W"], 240)
prm = O.params(wordsize=cfg["W"], mismatches=cfg["N"], margin=cfg["M"], iupac_mode=cfg["I"])
t = time.time()
ref = C.search(otable, seqs, prm, 16)
print("oracle", len(ref), f"{time.time() - t:.1f}s", flush=True)


def key(a):
    return set(zip(a["seq"].tolist(), a["pos1"].tolist(), a["rec"].tolist(), a["pos2"].tolist()))


R = key(ref)
for name, got in res.items():
    G = key(got)
    miss, extra = sorted(R - G), sorted(G - R)
    print(f"== {name}: missing {len(miss)} extra {len(extra)} identical={got.tobytes() == ref.tobytes()}")
    for lab, lst in (("missing", miss), ("extra", extra)):
        if not lst:
            continue
        h = {}
        for q, p1, _, _ in lst:
            b = (q, p1 >> 28)
            h[b] = h.get(b, 0) + 1
        print(lab, "by (seq, pos1>>28):", sorted(h.items()))
        print(lab, "first:", lst[:8], "last:", lst[-4:])
    # present-in-both per bin for context
    hb = {}
    for q, p1, _, _ in R:
        b = (q, p1 >> 28)
        hb[b] = hb.get(b, 0) + 1
    if name == "default":
        print("oracle by bin:", sorted(hb.items()))
