"""Time ablation variants of the scan kernel on the same resident c3 data (timing only).

Builds libmerpcr_hip_ablateN.so next to the product library from a copy of the sources
with timing-only variant N of scripts/ablate_variants.py applied (the product source has no
ablation code),
generates the workload once, and for each variant packs the genome, runs the
search `--steps` times and prints the mean scan-kernel time.  Hit counts of the
variants are meaningless except for variant 0 (the product kernel).
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0", help="0 = product, n = MP_ABLATE=n, NAME=VAL[+...] = defines, opt:name=val[,...] = search options, lib:path = a prebuilt library")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--no-build", action="store_true", help="use variant libraries built beforehand (CPU side)")
    ap.add_argument("--shard-of", type=int, default=1, help="search only rank 0's owned range of an N-way split")
    args = ap.parse_args()
    from merpcr_amd import _build
    variants = args.variants.split(",")
    libs = {}
    for v in variants:
        # 0 = product; n = MP_ABLATE=n; nt = non-temporal genome
        # stream; NAME=VAL[+NAME=VAL...] = those defines
        flags = None
        if v.startswith("lib:"):  # a library built beforehand (e.g. an earlier build's variant), path from the repo root
            libs[v] = os.path.join(ROOT, v[4:])
            continue
        if v == "0" or v.startswith("opt:"):
            defs = ()
        elif v == "atomopt":  # the compiler's atomic optimizer back on for mp_search.hip
            defs = ("MP_ATOMOPT=1",)
            flags = {}
        elif v == "nt":
            defs = ("MP_NT_STREAM=1",)
        elif "=" in v:
            defs = tuple(v.split("+"))
        else:  # a timing-only variant of scripts/ablate_variants.py on a copy of the sources
            defs = ()
        tag = "".join(ch if ch.isalnum() else "_" for ch in v)
        src_dir, src_tag = _build.CSRC, ""
        if v.isdigit() and v != "0":
            import ablate_variants
            src_dir = ablate_variants.make_source_dir(int(v), _build.CSRC,
                                                      os.path.join(tempfile.gettempdir(), f"mp_ablate_{v}"))
            src_tag = f"_ablate{v}"
        path = _build.LIB if v == "0" or v.startswith("opt:") else os.path.join(_build.LIBDIR, f"libmerpcr_hip_ablate{tag}.so")
        if args.no_build and os.path.exists(path):
            libs[v] = path
            continue
        saved = _build.SOURCE_FLAGS
        if flags is not None:
            _build.SOURCE_FLAGS = flags
        libs[v] = _build.build_native(defines=defs, lib=path, src_dir=src_dir, tag=src_tag)
        _build.SOURCE_FLAGS = saved
    if args.build_only:
        return
    import ctypes
    import torch
    from merpcr_amd import MerPCR, _native, synth
    cfg = dict(synth.CONFIGS[args.config])
    total = int(cfg["total"] * args.scale) // 64 * 64
    n_sts = max(1, int(cfg["n_sts"] * args.scale))
    sts = synth.make_sts(n_sts, W=cfg["W"], iupac=cfg["iupac"])
    dev = torch.device("cuda", 0)
    names, lens, buf, offs, planted = synth.build_genome_torch(
        total, cfg["records"], sts, seed=1, N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=dev)
    torch.cuda.synchronize()
    with tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False) as fh:
        fh.write(sts.text())
    out = {}
    for v in variants:
        lib = ctypes.CDLL(libs[v])
        _native._sig(lib)
        _native._lib = lib
        eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
        assert eng.load_sts_file(fh.name)
        table = eng.device_table()
        genome = _native.Genome(0, lens)
        for r, n in enumerate(lens):
            genome.put_device(r, buf.data_ptr() + int(offs[r]), n)
        genome.seal()
        s = _native.Search(table, genome)
        if v.startswith("opt:"):  # opt:name=int[,name=int...]: mp_search_set_options on the product library
            kw = {}
            for item in v[4:].split(","):
                k, val = item.split("=")
                kw[k] = val if k in ("tails", "sort", "generic") else int(val)
            s.set_options(**kw)
        from merpcr_amd.dist import shard_ranges
        rng = shard_ranges(lens, args.shard_of)[0] if args.shard_of > 1 else None
        s.run(rng)
        ms = []
        for _ in range(args.steps):
            n = s.run(rng)
            ms.append(s.last_stats()["scan_ms"])
        st = s.last_stats()
        out[v] = {"scan_ms": round(sum(ms) / len(ms), 3), "tail_ms": round(st["tail_ms"], 3), "pair_ms": round(st["pair_ms"], 3),
                  "hits": n, "candidates": st["candidates"], "survivors": st["survivors"]}
        if hasattr(lib, "mp_debug_pair_counts"):  # variant 52: cumulative over all runs
            pc = (ctypes.c_ulonglong * 8)()
            lib.mp_debug_pair_counts(pc)
            out[v]["pair_counts_cum"] = list(pc)
        print(f"variant {v}: {out[v]}", flush=True)
        s.close(); genome.close(); table.close()
        eng._dev_table = None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
