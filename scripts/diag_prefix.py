"""Diagnostic: one full-table prefix case (tests/test_gpu_fullscale.py) under several
search options / libraries, each compared with the C oracle: counts, duplicates, and the
first extra / missing hits."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from merpcr_amd import MerPCR, _native, synth  # noqa: E402
from oracle import c_oracle as C  # noqa: E402
from oracle import epcr_oracle as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
total = int(sys.argv[2]) if len(sys.argv) > 2 else 40_000_000
records = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cfg = synth.CONFIGS[name]
sts = synth.make_sts(cfg["n_sts"], W=cfg["W"], iupac=cfg["iupac"])
eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
with tempfile.TemporaryDirectory() as td:
    p = os.path.join(td, "c.sts")
    open(p, "w").write(sts.text())
    assert eng.load_sts_file(p)
table = eng.device_table()
dev = torch.device("cuda", 0)
names, lens, buf, offs, planted = synth.build_genome_torch(
    total, records, sts, seed=1, N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=dev)
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
genome = _native.Genome(0, lens)
for r, n in enumerate(lens):
    genome.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
genome.seal(stream)
host = buf.cpu().numpy()
seqs = [host[int(offs[r]):int(offs[r]) + lens[r]] for r in range(len(lens))]
otable = O.load_sts_lines(sts.text().splitlines(True), cfg["W"], 240)
prm = O.params(wordsize=cfg["W"], mismatches=cfg["N"], margin=cfg["M"], iupac_mode=cfg["I"])
ref = C.search(otable, seqs, prm, 16)
R = set(map(tuple, np.stack([ref["seq"], ref["pos1"], ref["pos2"], ref["rec"]], 1).tolist()))
print("oracle", len(ref), flush=True)
for label, opts in [("default", {}), ("tailkernel", dict(tails="kernel")),
                    ("inline", dict(tails="inline"))]:
    s = _native.Search(table, genome)
    if opts:
        s.set_options(**opts)
    got = s.fetch(s.run(None, stream))
    for rep in range(2):  # repeat: run-to-run determinism
        again = s.fetch(s.run(None, stream))
        if again.tobytes() != got.tobytes():
            print(label, "NONDETERMINISTIC run", rep, len(again), len(got))
    G = list(map(tuple, np.stack([got["seq"], got["pos1"], got["pos2"], got["rec"]], 1).tolist()))
    Gs = set(G)
    extra, miss = sorted(Gs - R), sorted(R - Gs)
    print(f"{label}: {len(got)} dup={len(G) - len(Gs)} extra={len(extra)} missing={len(miss)} identical={got.tobytes() == ref.tobytes()}",
          s.last_stats(), flush=True)
    if extra:
        print("  extra:", extra[:6])
    if miss:
        print("  missing:", miss[:6])
    s.close()
