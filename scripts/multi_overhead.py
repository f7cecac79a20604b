"""Host overhead of the one-process multi-device path (mp_multi_run, MerPCR(devices=...)):
wall time per call against the call's device span on devices[0] (mp_multi_timing: from
before the first search is enqueued to the gather's end).  Devices [0, 0] on a one-GPU box
(two owned halves searched on one device, gathered by device copies); a 1/8 c3 genome.
Prints one JSON line."""
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from merpcr_amd import MerPCR, _native, synth  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.125
devs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,0").split(",")]
cfg = synth.CONFIGS["c3"]
total = int(cfg["total"] * scale) // 64 * 64
sts = synth.make_sts(cfg["n_sts"], W=cfg["W"])
eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"])
with tempfile.TemporaryDirectory() as td:
    p = os.path.join(td, "c.sts")
    open(p, "w").write(sts.text())
    assert eng.load_sts_file(p)
table = eng.device_table()
names, lens, buf, offs, planted = synth.build_genome_torch(
    total, cfg["records"], sts, seed=1, N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=torch.device("cuda", 0))
host = buf.cpu().numpy()
m = _native.Multi(devs, [table] * len(devs))
m.genome(lens)
for r, n in enumerate(lens):
    m.put(r, host[int(offs[r]):int(offs[r]) + n])
m.seal()
ref_g = _native.Genome(0, lens)
for r, n in enumerate(lens):
    ref_g.put(r, host[int(offs[r]):int(offs[r]) + n])
ref_g.seal()
ref_s = _native.Search(table, ref_g)
want = ref_s.fetch(ref_s.run())
n = m.run()
got = m.fetch(n)
assert got.tobytes() == want.tobytes(), (len(got), len(want))
walls, spans, gathers = [], [], []
for _ in range(30):
    t = time.perf_counter()
    m.run()
    walls.append((time.perf_counter() - t) * 1e3)
    sp, g = m.timing()
    spans.append(sp)
    gathers.append(g)
single = []
for _ in range(30):
    t = time.perf_counter()
    ref_s.run()
    single.append((time.perf_counter() - t) * 1e3)
w, sp = np.array(walls), np.array(spans)
print(json.dumps({
    "devices": devs, "bases": int(total), "hits": int(n), "identical_to_single_device": True,
    "multi_run_wall_ms_median": round(float(np.median(w)), 4),
    "multi_run_span_ms_median": round(float(np.median(sp)), 4),
    "host_overhead_us_median": round(float(np.median(w - sp)) * 1e3, 1),
    "host_overhead_us_p90": round(float(np.percentile(w - sp, 90)) * 1e3, 1),
    "gather_ms_median": round(float(np.median(gathers)), 4),
    "single_device_whole_run_wall_ms_median": round(float(np.median(single)), 4),
    "note": "host overhead = wall time of mp_multi_run minus its device span on devices[0] (event before the "
            "first enqueue -> gather end); 30 calls after one checked call"}))
