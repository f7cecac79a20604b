"""Check that the synthetic c3 genome and the search are deterministic on the GPU."""
import hashlib
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from merpcr_amd import MerPCR, _native, synth

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
cfg = synth.CONFIGS["c3"]
total = int(cfg["total"] * scale) // 64 * 64
sts = synth.make_sts(int(cfg["n_sts"] * scale), W=11)
eng = MerPCR(wordsize=11, mismatches=1)
with tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False) as fh:
    fh.write(sts.text())
assert eng.load_sts_file(fh.name)
table = eng.device_table()
for trial in range(2):
    names, lens, buf, offs, planted = synth.build_genome_torch(total, 24, sts, 1, 1, 50, 11, 0.05, torch.device("cuda", 0))
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for o, n in zip(offs, lens):
        h.update(buf[int(o):int(o) + n].cpu().numpy().tobytes())
    g = _native.Genome(0, lens)
    for r, n in enumerate(lens):
        g.put_device(r, buf.data_ptr() + int(offs[r]), n)
    g.seal()
    s = _native.Search(table, g)
    res = [s.fetch(s.run()) for _ in range(3)]
    same = all(np.array_equal(res[0], x) for x in res[1:])
    print(f"trial {trial}: genome {h.hexdigest()[:16]} planted {planted} hits {len(res[0])} "
          f"repeat-identical {same} hitsha {hashlib.sha256(res[0].tobytes()).hexdigest()[:16]}", flush=True)
    del buf
