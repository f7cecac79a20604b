"""Benchmark: genome bases scanned per second (Gbp/s) + STS hits/s on MI355X.

Workload (BASELINE.json metric "W=11 N=1"; configs[2]):
  c3 = 100k synthetic STS primer pairs vs a 3 Gbp human-size synthetic genome
       (24 records), W=11 N=1 M=50, every STS planted in both orientations.
A step is one full pass of the hot path over the resident genome: seed scan +
primer verify + pair-check kernel, device ordering of the hits and the hit-count
readback (mp_search_run); for N > 1 also the RCCL gatherv of every rank's hits
to rank 0.  Inputs (seed table + packed genome) are resident in HBM before the
timed region.  Multi-GPU: one process per GPU.  Default --scaling weak: the job is
N genomes' worth of contigs, contig-sharded, one config-sized set of records per
rank (each rank's contigs drawn from its own seed), so per-GPU work is fixed and
`value` = all ranks' bases / the slowest rank's step time.  --scaling strong
splits ONE genome's (sequence, k) space into equal contiguous owned ranges.

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "genome bases scanned/sec (Gbp/s) + STS hits/sec, W=11 N=1, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip parameters)
BYTES_PER_BASE = 0.375       # 2-bit plane + 1-bit ambiguity plane, read once
BYTES_PER_HIT = 16           # 128-bit order key written per raw hit


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(workload: str):
    """HBM bytes per scan launch from the newest committed PMC pass of this workload
    (profiles/<tag>_pmc.json next to the bench line it was collected with), else None."""
    import glob
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")):
        tag = os.path.basename(f)[:-len("_pmc.json")]
        bj = os.path.join(ROOT, "profiles", f"{tag}_bench.json")
        try:
            if json.load(open(bj))["config"]["workload"] != workload:
                continue
            d = json.load(open(f))
        except (OSError, ValueError, KeyError):
            continue
        if "hbm_traffic_bytes_per_launch" in d and (best is None or os.path.getmtime(f) > best[0]):
            best = (os.path.getmtime(f), d["hbm_traffic_bytes_per_launch"], tag)
    return (best[1], best[2]) if best else (None, None)


def cpu_baseline(eng, names, lens, buf, offs, cfg, hits_dev, budget_s: float, threads: int):
    """Time the C oracle (scalar restatement, `threads` pthreads over k ranges) on whole
    leading records of the same genome, and check its hits against the GPU's."""
    import torch
    from oracle import c_oracle as C
    from oracle import epcr_oracle as O

    sts_lines = open(eng._sts_path).read().splitlines(True)
    table = O.load_sts_lines(sts_lines, cfg["W"], 240)
    prm = O.params(wordsize=cfg["W"], mismatches=cfg["N"], margin=cfg["M"], iupac_mode=cfg["I"])
    # calibrate on 64 Mbp of record 0
    probe = buf[int(offs[0]):int(offs[0]) + min(64_000_000, lens[0])].cpu().numpy()
    t = time.time()
    C.search(table, [probe], prm, threads)
    rate = len(probe) / max(time.time() - t, 1e-6)
    # whole leading records (exact T=1 semantics, so GPU and CPU hits must agree)
    nrec, nb = 0, 0
    while nrec < len(lens) and (nb == 0 or (nb + lens[nrec]) / rate <= budget_s):
        nb += lens[nrec]
        nrec += 1
    seqs = [buf[int(offs[r]):int(offs[r]) + lens[r]].cpu().numpy() for r in range(nrec)]
    t = time.time()
    ref = C.search(table, seqs, prm, threads)
    dt = time.time() - t
    mine = hits_dev[hits_dev["seq"] < nrec]
    parity = bool(len(mine) == len(ref) and mine.tobytes() == ref.tobytes())
    # the reference algorithm itself, as plain per-base Python (oracle/epcr_oracle.py), on 1 Mbp
    sub = probe[:1_000_000].tobytes().decode("ascii")
    t = time.time()
    O.scan_sequence(sub, table, prm)
    py_rate = len(sub) / (time.time() - t)
    return {
        "value": round(nb / dt / 1e9, 6), "unit": "Gbp/s", "cores": threads, "kind": "port",
        "sample": f"{nrec} whole leading record(s) = {nb / 1e6:.1f} Mbp of the same genome, same 100k-STS "
                  f"table, C restatement of engine.py:453-642 (oracle/epcr_oracle.c), {threads} thread(s)",
        "seconds": round(dt, 3), "hits": int(len(ref)),
        "parity_vs_gpu": parity,
        "reference_algorithm_python_mbps": round(py_rate / 1e6, 3),
    }


def end_to_end(eng, table, names, lens, buf, offs, device, stream):
    """One untimed-by-the-metric pass from host bytes to output text (SURVEY 8d t_e2e):
    H2D + 2-bit pack + exception index (mp_genome_put/seal), search, hit fetch and the
    native formatter.  Filtered FASTA bytes start in host memory, as after FASTA load."""
    import torch
    from merpcr_amd import _native
    from merpcr_amd.core.models import FASTARecord

    host = buf.cpu().numpy()
    recs = [FASTARecord(defline=">" + nm, sequence="", label=nm) for nm in names]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = _native.Genome(device, lens)
    for r, n in enumerate(lens):
        g.put(r, host[int(offs[r]):int(offs[r]) + n], stream=stream)
    g.seal(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    s = _native.Search(table, g)
    n = s.run(None, stream)
    hits = s.fetch(n)
    t2 = time.perf_counter()
    text = eng.format_bytes(recs, hits)
    t3 = time.perf_counter()
    s.close()
    g.close()
    bases = float(sum(lens))
    return {"seconds": round(t3 - t0, 3), "gbp_per_s": round(bases / (t3 - t0) / 1e9, 3),
            "upload_pack_s": round(t1 - t0, 3), "search_fetch_s": round(t2 - t1, 3),
            "format_s": round(t3 - t2, 3), "output_bytes": len(text),
            "note": "filtered sequence bytes in pageable host memory -> output text; PCIe-inclusive, "
                    "not the metric"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the config's genome and STS set")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = min(16, cores))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-bytes-to-output-text pass")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: each rank scans its own config-sized contig set (N x the genome); "
                         "strong: one genome split in N owned ranges")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic: time only rank 0's owned range of an N-way split on this one GPU "
                         "(no collective); the JSON line is then not the metric")
    args = ap.parse_args()

    import torch
    from merpcr_amd import MerPCR, _native, synth
    from merpcr_amd.dist import HIT_BYTES, gather_hits, shard_ranges

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    cfg = dict(synth.CONFIGS[args.config])
    total = int(cfg["total"] * args.scale) // 64 * 64
    n_sts = max(1, int(cfg["n_sts"] * args.scale))
    t_setup = time.time()
    sts = synth.make_sts(n_sts, W=cfg["W"], iupac=cfg["iupac"])
    eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"], device=local)
    with tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False) as fh:
        fh.write(sts.text())
        eng._sts_path = fh.name
    assert eng.load_sts_file(eng._sts_path)
    table = eng.device_table()
    weak = args.scaling == "weak"
    names, lens, buf, offs, planted = synth.build_genome_torch(
        total, cfg["records"], sts, seed=1 + (rank if weak else 0), N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=dev)
    torch.cuda.synchronize()
    genome = _native.Genome(local, lens)
    stream = torch.cuda.current_stream().cuda_stream
    t_pack = time.time()
    for r, n in enumerate(lens):
        genome.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
    genome.seal(stream)
    pack_s = time.time() - t_pack
    search = _native.Search(table, genome)
    if args.shard_of > 1:
        rng = shard_ranges(lens, args.shard_of)[0]
    elif weak:
        rng = None          # this rank's own contigs, whole
    else:
        rng = shard_ranges(lens, world)[rank]
    setup_s = time.time() - t_setup
    log(f"[rank {rank}] setup {setup_s:.1f}s (pack {pack_s:.2f}s) records={len(lens)} bases={sum(lens)} "
        f"sts={n_sts} recs={table.n_rec} planted={planted} table={table.stats()} genome={genome.stats()}")

    comm = None
    if world > 1:
        comm = torch.empty(1 << 20, dtype=torch.uint8, device=dev)

    def step():
        nonlocal comm
        n = search.run(rng, stream)
        if world > 1:
            need = max(n, 1) * HIT_BYTES
            if comm.numel() < need:
                comm = torch.empty(need * 2, dtype=torch.uint8, device=dev)
            search.fetch_device(comm.data_ptr(), comm.numel() // HIT_BYTES, stream)
            gather_hits(comm, n, seq_base=rank * len(lens) if weak else 0)
        return n

    for _ in range(args.warmup):
        step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scan_ms, tail_ms, pair_ms, order_ms, nhits = [], [], [], [], 0
    for _ in range(args.steps):
        nhits = step()
        ls = search.last_stats()
        scan_ms.append(ls["scan_ms"])
        tail_ms.append(ls["tail_ms"])
        pair_ms.append(ls["pair_ms"])
        order_ms.append(ls["order_ms"])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    st = search.last_stats()
    local_stats = torch.tensor([elapsed, float(nhits), float(st["windows"]), float(np.mean(scan_ms)),
                                float(sum(lens))],
                               dtype=torch.float64, device=dev)
    if world > 1:
        mx = local_stats.clone()
        torch.distributed.all_reduce(mx[:1], op=torch.distributed.ReduceOp.MAX)
        sm = local_stats.clone()
        torch.distributed.all_reduce(sm, op=torch.distributed.ReduceOp.SUM)
        elapsed = float(mx[0])
        tot_hits, tot_windows = float(sm[1]), float(sm[2])
        tot_bases = float(sm[4]) if weak else float(sum(lens))
    else:
        tot_hits, tot_windows = float(nhits), float(st["windows"])
        tot_bases = float(sum(lens))
    if rank != 0:
        torch.distributed.destroy_process_group()
        return
    bases = float(sum(lens))          # one rank's genome (= the whole job's at N=1 or strong)
    t_step = elapsed / args.steps
    kern_s = float(np.mean(scan_ms)) / 1e3
    alg_bytes = BYTES_PER_BASE * st["windows"] + BYTES_PER_HIT * nhits  # rank 0's scan launch
    achieved = alg_bytes / kern_s / 1e9 if kern_s > 0 else 0.0
    workload = (f"{args.config}: {n_sts} STS vs {bases / 1e9:.3f} Gbp ({len(lens)} records), "
                f"W={cfg['W']} N={cfg['N']} M={cfg['M']} I={cfg['I']}")
    if world > 1 and weak:
        workload += f" per rank ({world} contig sets, {tot_bases / 1e9:.3f} Gbp in all)"
    traffic, traffic_src = pmc_traffic(workload) if world == 1 else (None, None)
    out = {
        "metric": METRIC,
        "value": round(tot_bases / max(args.shard_of, 1) / t_step / 1e9, 4),
        "unit": "Gbp/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, merpcr_amd/synth.py; genome generated in HBM)",
        "config": {"workload": workload,
                   "sts": n_sts, "records": len(lens), "bases": int(bases), "W": cfg["W"], "N": cfg["N"],
                   "M": cfg["M"], "I": cfg["I"],
                   "parallelism": (f"contig shards x{world} (per-rank contig set, RCCL hit gatherv)" if weak
                                   else f"owned-k shards x{world} (RCCL hit gatherv)")},
        "hits": int(tot_hits),
        "hits_per_s": round(tot_hits / t_step, 1),
        "scan_kernel_ms": round(kern_s * 1e3, 3),
        "tail_kernel_ms": round(float(np.mean(tail_ms)), 3),
        "pair_kernel_ms": round(float(np.mean(pair_ms)), 3),
        "order_ms": round(float(np.mean(order_ms)), 3),
        "survivors": st["survivors"],
        "kernel_gbps_bases": round(st["windows"] / kern_s / 1e9, 3) if kern_s > 0 else None,
        "candidates": st["candidates"],
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": int(traffic) if traffic else None,
                     "traffic_source": f"profiles/{traffic_src}_pmc.json (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, "
                                       "gfx950-corrected; includes Infinity-Cache hits)" if traffic else None,
                     "kernel": "mp::dense_kernel" if cfg["W"] <= 9 else "mp::scan_kernel",
                     "alg_bytes_per_launch": int(alg_bytes)},
    }
    if args.shard_of > 1:
        out["diagnostic"] = f"rank 0 of a {args.shard_of}-way owned-range split, alone on one GPU (not the metric)"
    if world == 1 and not args.no_e2e:
        out["e2e"] = end_to_end(eng, table, names, lens, buf, offs, local, stream)
    if world == 1 and not args.no_cpu_baseline:
        hits = search.fetch(nhits)
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(eng, names, lens, buf, offs, cfg, hits, args.cpu_budget, threads)
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
