"""Where the CLI's end-to-end time goes (timing only): the c3 workload written as a FASTA
file, then `merpcr_amd.cli.main` run in-process under cProfile; prints the top functions
by cumulative time.  usage: python scripts/e2e_profile.py [--scale S]"""
import argparse
import cProfile
import os
import pstats
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    import torch
    from merpcr_amd import synth
    from merpcr_amd.cli import main as cli_main
    cfg = dict(synth.CONFIGS[args.config])
    total = int(cfg["total"] * args.scale) // 64 * 64
    sts = synth.make_sts(max(1, int(cfg["n_sts"] * args.scale)), W=cfg["W"], iupac=cfg["iupac"])
    names, lens, buf, offs, _ = synth.build_genome_torch(total, cfg["records"], sts, seed=1, N=cfg["N"], M=cfg["M"],
                                                         W=cfg["W"], nrun=cfg["nrun"], device=torch.device("cuda", 0))
    host = buf.cpu().numpy()
    del buf
    td = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    fa, st, out = os.path.join(td, "g.fa"), os.path.join(td, "s.sts"), os.path.join(td, "o.txt")
    with open(st, "w") as fh:
        fh.write(sts.text())
    with open(fa, "wb") as fh:
        for r, nm in enumerate(names):
            s = host[int(offs[r]):int(offs[r]) + lens[r]]
            fh.write(f">{nm} synthetic\n".encode())
            full = (len(s) // 60) * 60
            body = np.empty((full // 60, 61), dtype=np.uint8)
            body[:, :60] = s[:full].reshape(-1, 60)
            body[:, 60] = 10
            fh.write(body.tobytes())
            if len(s) > full:
                fh.write(s[full:].tobytes() + b"\n")
    del host
    argv = [st, fa, "-W", str(cfg["W"]), "-N", str(cfg["N"]), "-M", str(cfg["M"]), "-I", str(cfg["I"]), "-O", out]
    cli_main(argv)  # warm: HIP init, code objects
    pr = cProfile.Profile()
    t = time.time()
    pr.enable()
    rc = cli_main(argv)
    pr.disable()
    print(f"cli rc={rc} wall {time.time() - t:.3f}s, output {os.path.getsize(out)} bytes", flush=True)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
    for f in (fa, st, out):
        os.remove(f)
    os.rmdir(td)


if __name__ == "__main__":
    main()
