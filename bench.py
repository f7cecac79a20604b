"""Benchmark: genome bases scanned per second (Gbp/s) + STS hits/s on MI355X.

Workload (BASELINE.json metric "W=11 N=1"; configs[2]):
  c3 = 100k synthetic STS primer pairs vs a 3 Gbp human-size synthetic genome
       (24 records), W=11 N=1 M=50, every STS planted in both orientations.
A step is one full pass of the hot path over the resident genome: seed scan +
primer verify + pair-check kernels, device ordering of the hits and the hit-count
readback (mp_search_run); for N > 1 also the RCCL gatherv of every rank's hits
to rank 0 (mp_comm_gather_hits, inside the library).  Inputs (seed table + packed
genome) are resident in HBM before the timed region.  Multi-GPU: one process per
GPU; torch.distributed (gloo) is only the control plane (RCCL unique id, barrier,
max-over-ranks timing).  Default --scaling strong: ONE genome's (sequence, k) space
split into N equal owned ranges (the metric's "contig-sharded 1->8"); --scaling weak
gives every rank a config-sized contig set of its own.

Prints ONE JSON line on rank 0; exits 1 if the GPU hit list differs from the CPU
oracle's on the baseline sample.
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
N_SIMD, N_CU = 1024, 256     # MI355X: 256 CUs x 4 SIMD-32
L2_REQ_PEAK = 34.5e12 / 128  # L2 bandwidth / 128-B line (MI355X_MICROARCH.md, L2): ~270G requests/s


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores() -> int:
    """CPUs this job may use: the affinity mask, capped by a cgroup CPU quota if one is set."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    return n


def pmc_profile(workload: str, build: str):
    """Newest committed PMC summary of this workload taken with THIS build (profiles/<tag>_pmc.json
    whose "build" is the source digest of the library being benched, next to the bench line it
    was collected with; the highest tag wins), or (None, None).  A profile of another build is
    never used: its traffic would describe other kernels."""
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
        if d.get("build") != build:
            continue
        if "hbm_traffic_bytes_per_launch" in d and (best is None or tag > best[0]):
            best = (tag, d, tag)
    return (best[1], best[2]) if best else (None, None)


# Live counter passes (MI355X_MICROARCH.md, rocprofv3 section): per pass at most 8 SQ, 4 TCC
# (FETCH_SIZE takes 3, WRITE_SIZE 2) and 2 GRBM counters, and never a tracing domain beside --pmc.
PMC_PASSES = [
    ("fetch", ["FETCH_SIZE", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_LDS_IDX_ACTIVE",
               "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE"]),
    ("write", ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"]),
]


def pmc_counters(csv_path: str) -> dict:
    """Counter totals per search step from one rocprofv3 counter CSV: each dispatch's
    instances summed, the dispatches of each kernel form averaged (a list that overflowed
    and was rerun adds dispatches of the same form), and the forms of the step summed (a split
    W 7..9 table's step is two or three scan launches)."""
    import collections
    import csv
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(csv_path)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    by_form = collections.defaultdict(list)
    for (d, c), v in per.items():
        by_form[(names[d], c)].append(v)
    out = collections.defaultdict(float)
    for (_, c), v in by_form.items():
        out[c] += sum(v) / len(v)
    return dict(out)


def pmc_child_args(argv):
    """The caller's workload options for a counter pass, without its step counts and extras."""
    skip = {"--gpus", "--steps", "--warmup", "--cpu-budget", "--cpu-threads", "--handles", "--streams", "--depth"}
    flags = {"--no-cpu-baseline", "--no-e2e", "--no-ref-model", "--e2e-file", "--no-pmc", "--pmc-child"}
    child, i = [], 0
    while i < len(argv):
        a = argv[i]
        key = a.split("=")[0]
        if key in skip:
            i += 1 if "=" in a else 2
            continue
        if a not in flags:
            child.append(a)
        i += 1
    return child + ["--pmc-child", "--no-cpu-baseline", "--no-e2e", "--steps", "2", "--warmup", "1"]


def live_pmc(argv, kernel_regex: str, timeout_s: float = 150.0):
    """HBM traffic and issue counters of the scan stage measured in THIS bench invocation:
    rocprofv3 --pmc child passes of this script (--pmc-child: the same workload, build and
    options; setup and three searches, nothing else), one pass per counter set.  Returns
    (counters per step, note) or (None, reason)."""
    import glob
    import shutil
    import subprocess
    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if prof is None:
        return None, "rocprofv3 not found"
    child = pmc_child_args(argv)
    ctr = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for name, counters in PMC_PASSES:
            out = os.path.join(td, name)
            cmd = [prof, "--pmc", *counters, "--kernel-include-regex", kernel_regex, "-d", out, "-o", "run",
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), *child]
            t_pass = time.time()
            try:
                res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, cwd=td,
                                     env=dict(os.environ, TMPDIR=td))
            except subprocess.TimeoutExpired:
                return None, f"pass {name}: rocprofv3 timed out after {timeout_s:.0f} s"
            log(f"live counters: pass {name} took {time.time() - t_pass:.1f} s")
            if res.returncode:
                return None, f"pass {name}: rocprofv3 exit {res.returncode}: {res.stderr[-300:]}"
            files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
            if not files:
                return None, f"pass {name}: no counter CSV"
            for f in files:
                ctr.update(pmc_counters(f))
        # the scan stage's own duration: a kernel-trace pass (no counters) of the same child, one
        # handle so that no kernel of another step runs beside a scan (isolated dispatches)
        out = os.path.join(td, "trace")
        cmd = [prof, "--kernel-trace", "--kernel-include-regex", kernel_regex, "-d", out, "-o", "run",
               "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), *child,
               "--no-pipeline", "--steps", str(TRACE_STEPS)]
        t_pass = time.time()
        try:
            res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, cwd=td,
                                 env=dict(os.environ, TMPDIR=td))
        except subprocess.TimeoutExpired:
            return None, f"pass trace: rocprofv3 timed out after {timeout_s:.0f} s"
        log(f"live counters: pass trace took {time.time() - t_pass:.1f} s")
        if res.returncode:
            return None, f"pass trace: rocprofv3 exit {res.returncode}: {res.stderr[-300:]}"
        files = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)
        if not files:
            return None, "pass trace: no kernel-trace CSV"
        ctr.update(trace_stage_ns(files[0], kernel_regex))
    missing = [c for _, cs in PMC_PASSES for c in cs if c not in ctr]
    if missing:
        return None, f"counters missing from the passes: {missing}"
    return ctr, (f"live: {len(PMC_PASSES)} rocprofv3 --pmc passes and one --kernel-trace pass of this bench command "
                 f"(--pmc-child: same build, workload and options), kernels /{kernel_regex}/, per search step")


TRACE_STEPS = 8


def trace_stage_ns(csv_path: str, kernel_regex: str) -> dict:
    """The scan stage's duration per search step from a rocprofv3 kernel-trace CSV (the trace
    holds every kernel of the process; the stage's are those matching kernel_regex): each
    kernel form's dispatches averaged (the first dispatch of each form, a cold start, left out
    when there are more), the forms of a step summed (a split W 7..9 table scans two or three
    forms one after another).  The forms' dispatch counts and medians are kept beside it."""
    import collections
    import csv
    import re
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(csv_path)):
        if re.search(kernel_regex, r["Kernel_Name"]):
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total, forms = 0.0, {}
    for name, v in dur.items():
        use = v[1:] if len(v) > 1 else v
        total += sum(use) / len(use)
        forms[name] = {"dispatches": len(v), "mean_ns": round(sum(use) / len(use), 1),
                       "median_ns": float(np.median(use))}
    return {"_trace_stage_ns": total, "_trace_forms": forms}


def issue_bound(pmc: dict, dur_ns=None):
    """Issue-side utilisation of the dominant kernel from its committed PMC passes:
    VALU = SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) / (1024 SIMDs x kernel cycles),
    kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs); LDS = LDS-array cycles
    (SQ_LDS_IDX_ACTIVE) / (256 CUs x kernel cycles); the bank-conflict share of them; and the
    L2 request rate against the ~270G/s line ceiling (34.5 TB/s / 128 B)."""
    c = pmc.get("counters_mean_per_dispatch", pmc)
    out = {}
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if cyc > 0 and "SQ_INSTS_VALU" in c:
        out["valu_frac"] = round(c["SQ_INSTS_VALU"] * 2.0 / (N_SIMD * cyc), 4)
    if cyc > 0 and "SQ_LDS_IDX_ACTIVE" in c:
        out["lds_frac"] = round(c["SQ_LDS_IDX_ACTIVE"] / (N_CU * cyc), 4)
    if c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_ratio"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 4)
    if "SQ_WAIT_ANY" in c and c.get("SQ_WAVE_CYCLES"):
        out["wave_wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    req = c.get("TCC_REQ_sum") or (c.get("TCC_HIT_sum", 0.0) + c.get("TCC_MISS_sum", 0.0))
    dur = dur_ns or pmc.get("avg_duration_ns_trace_isolated") or pmc.get("avg_duration_ns_trace")
    if req and dur:
        out["l2_req_per_launch"] = int(req)
        out["l2_req_frac"] = round(req / (dur * 1e-9) / L2_REQ_PEAK, 4)
    return out


def roofline_time(pmc, events_s: float):
    """The scan stage's time for the roofline (seconds) and where it came from: the isolated
    dispatches of this command's own kernel-trace pass (rocprofv3's clock, no event between
    kernels); else a committed profile's isolated mean; else the HIP events (no trace ran: N > 1,
    a shard, --no-pmc).  A profile's mean over every dispatch never stands in: it includes the
    pipelined steps' overlapped scans (c3 3.16 ms against 2.06 isolated)."""
    pmc = pmc or {}
    if pmc.get("_trace_stage_ns"):
        return pmc["_trace_stage_ns"] / 1e9, ("rocprofv3 --kernel-trace pass of this command: mean isolated "
                                              "dispatch of each scan form, forms of a step summed")
    if pmc.get("avg_duration_ns_trace_isolated"):
        return pmc["avg_duration_ns_trace_isolated"] / 1e9, "avg_duration_ns_trace_isolated of the committed profile"
    return events_s, "HIP events (no trace pass)"


def agreed_comm(local: int, rank: int, world: int):
    """The RCCL communicator (merpcr_amd.dist.native_comm), or None on every rank when any
    rank could not make one: the job then gathers over gloo on the host (slower, same list)
    instead of failing.  Collective."""
    import torch.distributed as dist
    from merpcr_amd.dist import native_comm
    comm, err = None, None
    try:
        comm = native_comm(local)
    except Exception as e:  # noqa: BLE001 (reported, then every rank takes the same path)
        err = f"{type(e).__name__}: {e}"
    errs = [None] * world
    dist.all_gather_object(errs, err)
    if any(errs):
        log(f"[rank {rank}] RCCL communicator unavailable ({[x for x in errs if x][0]}); host gather")
        if comm is not None:
            comm.close()
        return None
    return comm


def cpu_baseline(eng, lens, buf, offs, cfg, hits_dev, budget_s: float, threads: int):
    """Time the C oracle (scalar restatement, `threads` pthreads over k ranges) on whole
    leading records of the same genome, and check its hits against the GPU's."""
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
    return {
        "value": round(nb / dt / 1e9, 6), "unit": "Gbp/s", "cores": threads, "kind": "port",
        "sample": f"{nrec} whole leading record(s) = {nb / 1e6:.1f} Mbp of the same genome, same STS "
                  f"table, C restatement of engine.py:453-642 (oracle/epcr_oracle.c), {threads} thread(s) "
                  f"= every CPU this job may use (affinity mask and cgroup quota)",
        "seconds": round(dt, 3), "hits": int(len(ref)),
        "parity_vs_gpu": parity,
    }, table, prm


def reference_model(table, prm, buf, offs, lens, cores: int, budget_s: float):
    """The reference's own execution model at -T <cores> (engine.py:380-434): the Python
    restatement of the scan (oracle/epcr_oracle.py) over the reference's chunk plan of a
    record prefix, one ProcessPool worker per chunk receiving the pickled table, pool start
    included as in the reference.  The prefix is sized to ~budget_s from a one-core
    calibration (no extrapolation: the figure is the measured prefix)."""
    import concurrent.futures
    import multiprocessing
    from oracle import epcr_oracle as O

    rec0 = buf[int(offs[0]):int(offs[0]) + lens[0]]
    probe = rec0[:200_000].cpu().numpy().tobytes().decode("ascii")
    t = time.time()
    O.scan_sequence(probe, table, prm)
    rate1 = len(probe) / max(time.time() - t, 1e-6)
    n = int(min(100_000_000, lens[0], rate1 * cores * budget_s))
    seq = rec0[:n].cpu().numpy().tobytes().decode("ascii")
    plan = O.chunk_plan(n, cores, table.max_pcr_size, prm["margin"])
    tasks = [(seq[o:o + ln], o, table, prm) for o, ln in plan]
    t = time.time()
    with concurrent.futures.ProcessPoolExecutor(max_workers=len(plan),
                                                mp_context=multiprocessing.get_context("spawn")) as ex:
        hits = sum(len(h) for h in ex.map(O.scan_chunk, tasks))
    dt = time.time() - t
    return {"value": round(n / dt / 1e6, 3), "unit": "Mbp/s", "cores": len(plan), "kind": "port",
            "sample": f"first {n / 1e6:.1f} Mbp of record 0, {len(plan)} chunks (-T {cores} plan, engine.py:380-410), "
                      f"one spawned worker per chunk, the table pickled into every task as the reference's bound-method submit does, pure-Python scan "
                      f"(oracle/epcr_oracle.py restating engine.py:453-642)",
            "seconds": round(dt, 3), "hits_with_chunk_duplicates": int(hits),
            "one_core_mbps": round(rate1 / 1e6, 3)}


def in_range(hits, rng):
    """Mask of the hits whose (seq, pos1) lies in the owned range (seq_begin, seq_end, k_begin, k_end)."""
    sb, se, kb, ke = rng
    q, k = hits["seq"].astype(np.int64), hits["pos1"].astype(np.int64)
    after_lo = (q > sb) | ((q == sb) & (k >= kb))
    before_hi = (q < se) | ((q == se) & (k < ke))
    return after_lo & before_hi


def parity_distributed(table, genome, search, rng, got, world, rank, weak, n_seq, stream):
    """Correctness gate of a sharded or multi-rank run (the oracle gate covers N=1):
    * every rank: its own sorted list (seq shifted as the gather shifts it) is hashed, and
      rank 0 compares each rank's segment of the gathered list with that rank's hash;
    * strong scaling / --shard-of: rank 0's single-device search of the WHOLE genome
      (itself checked against the C oracle by the N=1 bench) must equal the gathered
      list, or, for a shard, its owned slice."""
    import hashlib
    from merpcr_amd import _native
    mine = search.fetch(search.last_hits(), stream).copy()
    if weak:
        mine["seq"] += n_seq * rank
    digest = hashlib.sha256(mine.tobytes()).hexdigest()
    ok, why = True, []
    if world > 1:
        import torch.distributed as dist
        every = [None] * world
        dist.all_gather_object(every, (len(mine), digest))
        if rank == 0:
            off = 0
            for r, (n, d) in enumerate(every):
                seg = got[off:off + n] if got is not None else None
                if seg is None or len(seg) != n or hashlib.sha256(seg.tobytes()).hexdigest() != d:
                    ok = False
                    why.append(f"rank {r} segment differs")
                off += n
            if got is not None and off != len(got):
                ok = False
                why.append(f"gathered {len(got)} hits, ranks hold {off}")
    if rank == 0 and not weak:
        full_s = _native.Search(table, genome)
        full = full_s.fetch(full_s.run(None, stream), stream)
        full_s.close()
        if world > 1:
            if got is None or got.tobytes() != full.tobytes():
                ok = False
                why.append(f"gathered list ({None if got is None else len(got)}) != single-device "
                           f"whole-genome list ({len(full)})")
        if rng is not None and world == 1:
            want = full[in_range(full, rng)]
            if mine.tobytes() != want.tobytes():
                ok = False
                why.append(f"shard list ({len(mine)}) != the owned slice of the whole-genome list ({len(want)})")
    return {"ok": ok, "checked": ("gathered list vs per-rank hashes" if world > 1 else "") +
            ("" if weak else (" + " if world > 1 else "") + "vs rank 0's single-device whole-genome search"),
            "problems": why}


def end_to_end(eng, table, names, lens, buf, offs, device, stream):
    """One pass from host bytes to output text (SURVEY 8d t_e2e), not the metric:
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


def end_to_end_file(sts_path, names, lens, buf, offs, cfg, device):
    """The CLI from files: the genome written as FASTA (60-column lines), then
    `python -m merpcr_amd sts fasta -O out` timed in a child process: FASTA parse
    (mp_fasta_load), upload + pack, search, format and write.  Not the metric."""
    import subprocess
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        fa = os.path.join(td, "g.fa")
        t = time.time()
        with open(fa, "wb") as fh:
            for r, nm in enumerate(names):
                s = buf[int(offs[r]):int(offs[r]) + lens[r]].cpu().numpy()
                fh.write(f">{nm} synthetic\n".encode())
                full = (len(s) // 60) * 60
                body = np.empty((full // 60, 61), dtype=np.uint8)
                body[:, :60] = s[:full].reshape(-1, 60)
                body[:, 60] = 10
                fh.write(body.tobytes())
                if len(s) > full:
                    fh.write(s[full:].tobytes() + b"\n")
        write_s = time.time() - t
        out = os.path.join(td, "hits.txt")
        cmd = [sys.executable, "-m", "merpcr_amd", sts_path, fa, "-W", str(cfg["W"]), "-N", str(cfg["N"]),
               "-M", str(cfg["M"]), "-I", str(cfg["I"]), "-O", out, "--device", str(device)]
        t = time.time()
        res = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
        dt = time.time() - t
        if res.returncode:
            log(res.stderr[-2000:])
            return {"error": f"CLI exit {res.returncode}"}
        lines = sum(1 for _ in open(out, "rb"))
        size = os.path.getsize(fa)
    return {"seconds": round(dt, 3), "gbp_per_s": round(sum(lens) / dt / 1e9, 3), "fasta_bytes": size,
            "hit_lines": lines, "fasta_write_s": round(write_s, 3),
            "note": "python -m merpcr_amd on a 60-column FASTA file to an output file, child process wall "
                    "time (interpreter start, FASTA parse, upload + pack, search, format, write); not the metric"}


def free_port() -> int:
    """A TCP port on 127.0.0.1 that nothing listens on right now (the child job's rendezvous)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launcher_command(argv, n: int, port: int):
    """The one-rank-per-GPU job `bench.py --gpus N` starts for itself when it was not launched
    by torch.distributed.run: the same arguments, N local ranks, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def resolve_world(gpus, env) -> tuple:
    """(ranks, launch): how many ranks the job has and whether this process must start them.
    WORLD_SIZE set (torch.distributed.run): it is the rank count, and an explicit --gpus must
    agree with it.  Unset: --gpus N > 1 means launch N ranks as a child job; 1 (or no flag) is
    the single-process N=1 bench."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if gpus is not None and int(ws) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (launched with "
                             f"{ws} ranks); pass the same N to both or drop --gpus")
        return int(ws), False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {n}")
    return n, n > 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); N > 1 without torch.distributed.run launches "
                         "the N-rank job itself (default: WORLD_SIZE, else 1)")
    # 20 timed steps: the pipeline fills at the first and drains at the last, which 5 steps
    # carried as ~2% of c3's step (2.068 against 2.015-2.03 ms with 10-20 steps)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the config's genome and STS set")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = every usable CPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ref-model", action="store_true", help="skip the Python ProcessPool (-T) line")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-bytes-to-output-text pass")
    ap.add_argument("--e2e-file", action="store_true", help="also time the CLI from a FASTA file")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong: one genome split in N owned ranges; weak: each rank scans its own "
                         "config-sized contig set (N x the genome)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="diagnostic: every rank on device 0 (rehearses the N-rank path, RCCL included, on a "
                         "one-GPU box); the JSON line is then not the metric")
    ap.add_argument("--gather", default="ipc", choices=["ipc", "rccl", "host"],
                    help="N > 1: the per-step hit gather to rank 0 -- ipc: copy-engine puts into rank 0's "
                         "regions (IpcGather, no kernel on the CUs); rccl: mp_comm_gather_hits; host: gloo")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one search handle: every step waits for the previous one (no run queued ahead)")
    ap.add_argument("--handles", type=int, default=4,
                    help="search handles of the pipeline")
    ap.add_argument("--streams", type=int, default=0,
                    help="streams the handles are dealt onto round-robin (0: one per handle); with fewer "
                         "streams than handles a stream runs step i's tail/pair/order then step i+streams' scan "
                         "(round 6, same box: one per handle 1/8 c3 0.293-0.295 ms against 0.301-0.305 on 2 "
                         "streams, c4 2.649-2.654 against 2.692; profiles/r06n_streams_ab.json)")
    ap.add_argument("--depth", type=int, default=2,
                    help="steps enqueued ahead of the one the host completes (1: step i+1 is enqueued before "
                         "the host waits for step i); at most handles - 1")
    ap.add_argument("--one-stream", action="store_true",
                    help="pipelined handles share one stream (no kernel of step i+1 overlaps step i)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic: time only rank 0's owned range of an N-way split on this one GPU "
                         "(no collective); the JSON line is then not the metric")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 counter passes (roofline.traffic / issue)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)  # live_pmc's passes
    ap.add_argument("--opts", default="",
                    help="diagnostic A/B: search options for every handle, name=value[,...] (_native.Search.set_options)")
    args = ap.parse_args()
    # N > 1 and no launcher: start the N-rank job as a child before anything touches the GPU
    # (this process never initialises HIP), and exit with its code
    world, launch = resolve_world(args.gpus, os.environ)
    if launch:
        import subprocess
        cmd = launcher_command(sys.argv[1:], world, free_port())
        log("launching: " + " ".join(cmd))
        sys.exit(subprocess.call(cmd, cwd=ROOT))

    import torch
    from merpcr_amd import MerPCR, _native, synth
    from merpcr_amd.dist import HIT_BYTES, native_comm, shard_ranges

    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = None
    gmode = args.gather if world > 1 else None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")          # control plane only
        # data plane (--gather): copy-engine puts into rank 0's HBM (default), or RCCL inside
        # libmerpcr_hip (RCCL refuses two ranks on one device: a one-GPU rehearsal asking for
        # it gathers through gloo on the host instead)
        if gmode == "rccl" and args.rehearse_one_gpu:
            gmode = "host"
        comm = agreed_comm(local, rank, world) if gmode == "rccl" else None
        if gmode == "rccl" and comm is None:
            gmode = "host"

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
        total, cfg["records"], sts, seed=1 + (rank if weak else 0), N=cfg["N"], M=cfg["M"], W=cfg["W"],
        nrun=cfg["nrun"], device=dev)
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
    elif weak or world == 1:
        rng = None          # this rank's own contigs / the whole genome
    else:
        rng = shard_ranges(lens, world)[rank]
    setup_s = time.time() - t_setup
    log(f"[rank {rank}] setup {setup_s:.1f}s (pack {pack_s:.2f}s) records={len(lens)} bases={sum(lens)} "
        f"sts={n_sts} recs={table.n_rec} planted={planted} table={table.stats()} split={table.split()} genome={genome.stats()} "
        f"range={rng}")

    gathered = None
    last_gloo = [None]  # host gather: the host-gathered bytes of the last step
    if gmode == "rccl":
        gathered = torch.empty((1 << 22) * HIT_BYTES, dtype=torch.uint8, device=dev)  # rank 0's gather buffer
    shift = len(lens) * rank if weak else 0
    # Pipeline: 4 handles, each on its own stream, step i+2 enqueued before the host completes
    # step i.  Step i+1's scan takes the CUs as step i's scan blocks leave, so step i's chain
    # (tail, pair, order) runs after it; with 2 handles the host enqueued step i+2 only after
    # completing step i, which left ~13 us of idle GPU between the chains and the next scan
    # (1/8 c3 0.303-0.306 -> 0.294-0.295 ms queued two ahead, profiles/r06j_pipeline_ab.json).
    # With the 4 handles on 2 streams step i+2's scan still queued behind step i's chain; on
    # their own streams it starts on the CUs the latency-bound chains leave idle: 1/8 c3
    # 0.301-0.305 -> 0.293-0.295 ms, c4 2.692 -> 2.649-2.654 ms, c3 2.046-2.051 -> 2.028-2.043
    # (profiles/r06n_streams_ab.json).
    nbuf = 1 if args.no_pipeline else max(2, args.handles)
    ipcg = None
    if gmode == "ipc":
        # regions of twice the largest rank's hit count (one untimed run to learn it); every
        # rank must map rank 0's buffers, else the job falls back to RCCL (or the host gather)
        from merpcr_amd.dist import IpcGather
        n0 = search.run(rng, stream)
        every = [None] * world
        dist.all_gather_object(every, n0)
        err = None
        try:
            ipcg = IpcGather(local, max(4096, 2 * max(every)), slots=nbuf)  # a region slot per handle
            ipcg.put(search, stream)  # a probe put of that run: the copy engines reach rank 0's HBM
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 (reported, then every rank takes the same fallback)
            err = f"{type(e).__name__}: {e}"
        dist.barrier()
        if err is None and rank == 0 and ipcg.counts() != every:
            err = f"probe put: rank 0 read counts {ipcg.counts()}, the ranks wrote {every}"
        errs = [None] * world
        dist.all_gather_object(errs, err)
        if any(errs):
            log(f"[rank {rank}] IPC gather unavailable ({[x for x in errs if x][0]}); falling back")
            if ipcg is not None:
                ipcg.close()
            ipcg = None
            gmode = "host" if args.rehearse_one_gpu else "rccl"
            if gmode == "rccl":
                comm = agreed_comm(local, rank, world)
                if comm is None:
                    gmode = "host"
                else:
                    gathered = torch.empty((1 << 22) * HIT_BYTES, dtype=torch.uint8, device=dev)

    # Steps are pipelined two deep (mp_search_enqueue / mp_search_complete on two search
    # handles over the same resident table and genome): step i+1's kernels are queued before
    # the host waits for step i, so the host turnaround between runs is off the GPU's path.
    # With N > 1 each completed step's RCCL gather runs on a stream of its own, and the
    # handle's next run waits (on the device) for its gather to have sent the hits.
    handles = [search] + [_native.Search(table, genome) for _ in range(nbuf - 1)]
    if args.opts:
        kw = {}
        for item in args.opts.split(","):
            k, val = item.split("=")
            kw[k] = val if k in ("tails", "sort", "generic") else (val.lower() in ("1", "true") if k in (
                "defer", "dense", "rank_filter", "split", "ref32") else int(val))
        for h in handles:
            h.set_options(**kw)
    # one stream per handle (--one-stream: all on the default stream): step i+1's scan may then
    # start on the CUs that step i's latency-bound tail / pair / order kernels leave idle
    nstr = nbuf if args.streams <= 0 else max(1, min(args.streams, nbuf))
    own = [torch.cuda.current_stream()] + [
        torch.cuda.current_stream() if args.one_stream else torch.cuda.Stream(device=dev) for _ in range(nstr - 1)]
    streams = [own[j % nstr] for j in range(nbuf)]  # handle j's stream
    depth = max(1, min(args.depth, nbuf - 1)) if nbuf > 1 else 1
    log(f"[rank {rank}] pipeline: {nbuf} handles on {nstr} streams, {depth} step(s) ahead")
    gstream = torch.cuda.Stream(device=dev) if comm is not None else None
    gdone = [None] * nbuf
    scan_ms = []

    def gather(h, j):
        """Every rank's hits of handle h's completed run to rank 0; the job's hit count (this
        rank's under --gather ipc: rank 0 reads the counts after the steps)."""
        nonlocal gathered
        n = h.last_hits()
        if world == 1:
            return n, None
        if ipcg is not None:  # on the handle's stream, into the handle's own region slot
            ipcg.put(h, streams[j].cuda_stream, slot=j)
            return n, None
        if comm is None:  # host gather over gloo
            from merpcr_amd.dist import gather_hits as gloo_gather
            mine = h.fetch(n, stream)
            buf_h = torch.from_numpy(np.frombuffer(mine.tobytes() + b"\0" * HIT_BYTES, dtype=np.uint8).copy())
            got = gloo_gather(buf_h, n, seq_base=shift)
            last_gloo[0] = got
            return (got.numel() // HIT_BYTES if rank == 0 else n), None
        cap = gathered.numel() // HIT_BYTES if rank == 0 else 0
        try:
            n = comm.gather_hits(h, gathered.data_ptr(), cap, shift, gstream.cuda_stream)
        except _native.NativeError as e:
            if e.code != _native.MP_E_CAP:
                raise
            # rank 0's buffer too small: every rank got MP_E_CAP; grow and gather again
            gstream.synchronize()
            gathered = torch.empty(comm.last_total * 2 * HIT_BYTES, dtype=torch.uint8, device=dev)
            cap = gathered.numel() // HIT_BYTES if rank == 0 else 0
            n = comm.gather_hits(h, gathered.data_ptr(), cap, shift, gstream.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(gstream)
        return n, ev

    def finish(j):
        h = handles[j]
        h.complete()
        sm = h.last_stats()["scan_ms"]
        if sm >= 0:
            scan_ms.append(sm)
        n, gdone[j] = gather(h, j)
        return n

    def run_steps(k):
        """k steps, pipelined: step i is enqueued, then the host completes step i - depth;
        returns the last step's job-wide hit count."""
        import collections
        pend, total = collections.deque(), 0
        for i in range(k):
            j = i % nbuf
            if j in pend:  # handle j still holds a run: complete everything up to it
                while pend:
                    q = pend.popleft()
                    total = finish(q)
                    if q == j:
                        break
            if gdone[j] is not None:  # its previous run's hits are still being sent
                streams[j].wait_event(gdone[j])
                gdone[j] = None
            handles[j].enqueue(rng, streams[j].cuda_stream)
            pend.append(j)
            while len(pend) > depth:
                total = finish(pend.popleft())
        while pend:
            total = finish(pend.popleft())
        return total

    # Timed steps: no per-stage events (each idles the GPU ~6 us).  The scan kernel's own two
    # events (roofline.achieved: HIP events on its launch stream) stay in the timed steps only
    # when no kernel of another step can run beside it (one stream, N = 1): with two streams
    # step i+1's scan overlaps step i's tail / pair / order, and the events would time both.
    # Otherwise the scan is timed in three untimed steps after the timed ones, one at a time
    # on one stream, on the same resident data.
    scan_in_timed = (nbuf == 1 or args.one_stream) and world == 1 and args.shard_of <= 1
    for h in handles:
        h.set_stage_timing(False)
        h.set_scan_timing(scan_in_timed)
    # every handle runs once before the warmup: a handle's first run of a range uploads its span
    # table and waits for its stream, which must not fall inside the timed steps (with more
    # handles than warmup steps it did: 4 handles, 2 warmup steps, c3 2.05 -> 4.0 ms per step)
    for j, h in enumerate(handles):
        h.enqueue(rng, streams[j].cuda_stream)
        finish(j)
    torch.cuda.synchronize()
    run_steps(args.warmup)
    scan_ms.clear()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nhits = run_steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if ipcg is not None:  # every rank's puts are complete (synchronised before the barrier)
        if ipcg.settle():  # a put did not fit its region: regrown, every slot put again (untimed)
            log(f"[rank {rank}] IPC gather regions regrown to {ipcg.cap} hits")
        if rank == 0:
            nhits = int(sum(ipcg.counts((args.steps - 1) % nbuf)))
    timed_scan_ms = list(scan_ms)
    if args.pmc_child:  # a counter pass of live_pmc: the counters are all it is for
        for h in handles:
            h.close()
        print(json.dumps({"pmc_child": True, "runs": args.warmup + args.steps}), flush=True)
        return
    # single-search latency beside the pipelined step: handle 0 alone, each run enqueued only
    # after the previous one completed (host turnaround included, no events), median of 5
    single_ms = None
    if world == 1:
        torch.cuda.synchronize()
        search.set_scan_timing(False)
        search.set_stage_timing(False)
        lat = []
        for _ in range(5):
            t1 = time.perf_counter()
            search.enqueue(rng, stream)
            search.complete()
            lat.append(time.perf_counter() - t1)
        single_ms = float(np.median(lat)) * 1e3
    # untimed: three more steps of handle 0 alone (the scan time when the timed steps carried
    # no events), the last with every stage timed (the stage breakdown)
    torch.cuda.synchronize()
    for j in range(nbuf):
        gdone[j] = None
    search.set_scan_timing(True)
    scan_ms.clear()
    for u in range(3):
        search.set_stage_timing(u == 2)
        search.enqueue(rng, stream)
        finish(0)
        torch.cuda.synchronize()
        gdone[0] = None
    if not timed_scan_ms:
        timed_scan_ms = list(scan_ms)
    scan_ms = timed_scan_ms
    stages = search.last_stats()
    tail_ms, pair_ms, order_ms = [stages["tail_ms"]], [stages["pair_ms"]], [stages["order_ms"]]
    st = search.last_stats()
    for h in handles[1:]:
        h.close()
    if world > 1:
        mx = torch.tensor([elapsed], dtype=torch.float64)
        torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX)
        sm = torch.tensor([float(sum(lens))], dtype=torch.float64)
        torch.distributed.all_reduce(sm)
        elapsed = float(mx[0])
        tot_bases = float(sm[0]) if weak else float(sum(lens))
    else:
        tot_bases = float(sum(lens))
    tot_hits = float(nhits)  # after the gather: every rank's hits (N > 1)
    dist_check = None
    if world > 1 or args.shard_of > 1:
        got = None
        if ipcg is not None:  # collective: the untimed steps' puts (slot 0) may need a regrow too
            torch.cuda.synchronize()
            torch.distributed.barrier()
            ipcg.settle()
        if world > 1 and rank == 0:
            if ipcg is not None:
                raw = ipcg.hits([len(lens) * r for r in range(world)] if weak else None).cpu().numpy()
            else:
                raw = (gathered[:nhits * HIT_BYTES] if comm is not None else last_gloo[0]).cpu().numpy()
            got = np.frombuffer(raw.tobytes(), dtype=_native.HIT_DTYPE)
        dist_check = parity_distributed(table, genome, search, rng, got, world, rank, weak, len(lens), stream)
    if ipcg is not None:  # every rank unmaps before rank 0's buffers go
        ipcg.close()
        torch.distributed.barrier()
    if rank != 0:
        if comm is not None:
            comm.close()
        torch.distributed.destroy_process_group()
        return
    bases = float(sum(lens))          # one rank's genome (= the whole job's at N=1 or strong)
    t_step = elapsed / args.steps
    kern_ev_s = float(np.mean(scan_ms)) / 1e3  # HIP events on the scan's launch stream
    alg_bytes = BYTES_PER_BASE * st["windows"] + BYTES_PER_HIT * search.last_hits()  # rank 0's scan launch
    # the scan stage's kernels (events around all of them): a split W 7..9 table scans its two
    # exact seeds with scan_kernel (plus dense_kernel over the records they cannot carry)
    sp = table.split()
    if sp["seed_tables"]:
        W = cfg["W"]
        scan_label = (f"mp::scan_kernel x{sp['seed_tables']} (split seeds: exact [0, 11)"
                      + (f" + gapped [0, {W}) ++ [11, {22 - W})" if sp["seed_tables"] > 1 else "")
                      + (f" + dense_kernel over {sp['rest_records']} records" if sp["rest_records"] else "")
                      + "; one stage, HIP events around all of it)")
    else:
        scan_label = "mp::dense_kernel" if cfg["W"] <= 9 else "mp::scan_kernel"
    workload = (f"{args.config}: {n_sts} STS vs {bases / 1e9:.3f} Gbp ({len(lens)} records), "
                f"W={cfg['W']} N={cfg['N']} M={cfg['M']} I={cfg['I']}")
    if world > 1 and weak:
        workload += f" per rank ({world} contig sets, {tot_bases / 1e9:.3f} Gbp in all)"
    gather_label = {"ipc": "hit gather: copy-engine puts into rank 0's HBM over xGMI",
                    "rccl": "RCCL hit gatherv", "host": "hit gather through the host (gloo)"}.get(
        gmode, f"N > 1 hit gather: --gather {args.gather}")
    from merpcr_amd._build import source_digest
    build = source_digest()
    # roofline.traffic / issue: counters measured now, in child passes of this very command;
    # failing that, a committed profile of this same build; else null with the reason
    pmc, pmc_src, traffic, why = None, None, None, "not measured for N > 1 or shard runs"
    if world == 1 and args.shard_of <= 1:
        regex = "scan_kernel|dense_kernel" if (sp["seed_tables"] or cfg["W"] <= 9) else "scan_kernel"
        live, why = (None, "--no-pmc") if args.no_pmc else live_pmc(sys.argv[1:], regex)
        if live is not None:
            pmc, pmc_src = live, why
            traffic = 2.0 * live["FETCH_SIZE"] * 1024 + live["WRITE_SIZE"] * 1024
        else:
            log(f"live counters unavailable ({why}); looking for a committed profile of build {build}")
            prof, tag = pmc_profile(workload, build)
            if prof is not None:
                pmc, pmc_src = prof, f"profiles/{tag}_pmc.json (committed profile of this build)"
                traffic = prof["hbm_traffic_bytes_per_launch"]
    kern_s, kern_src = roofline_time(pmc, kern_ev_s)
    achieved = alg_bytes / kern_s / 1e9 if kern_s > 0 else 0.0
    out = {
        "metric": METRIC,
        "value": round(tot_bases / max(args.shard_of, 1) / t_step / 1e9, 4),
        "unit": "Gbp/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 3),
        "single_run_ms": round(single_ms, 3) if single_ms is not None else None,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, merpcr_amd/synth.py; genome generated in HBM)",
        "config": {"workload": workload,
                   "sts": n_sts, "records": len(lens), "bases": int(bases), "W": cfg["W"], "N": cfg["N"],
                   "M": cfg["M"], "I": cfg["I"],
                   "parallelism": (f"contig sets x{world} (one per rank, {gather_label})" if weak
                                   else f"owned (sequence, k) ranges x{world} of one genome ({gather_label})")},
        "hits": int(tot_hits),
        "hits_per_s": round(tot_hits / t_step, 1),
        "scan_kernel_ms": round(kern_s * 1e3, 3),
        "scan_kernel_ms_source": kern_src,
        "scan_kernel_ms_events": round(kern_ev_s * 1e3, 3),
        "tail_kernel_ms": round(float(np.mean(tail_ms)), 3),
        "pair_kernel_ms": round(float(np.mean(pair_ms)), 3),
        "order_ms": round(float(np.mean(order_ms)), 3),
        "survivors": st["survivors"],
        "kernel_gbps_bases": round(st["windows"] / kern_s / 1e9, 3) if kern_s > 0 else None,
        "candidates": st["candidates"],
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": int(traffic) if traffic else None,
                     "traffic_source": (pmc_src + "; 2 x FETCH_SIZE KiB (gfx950 half-count) + WRITE_SIZE KiB, "
                                        "Infinity-Cache hits included") if traffic else None,
                     "traffic_null_reason": None if traffic else why,
                     "kernel": scan_label,
                     "alg_bytes_per_launch": int(alg_bytes),
                     "time_ms": round(kern_s * 1e3, 4),
                     "time_source": kern_src,
                     "trace_forms": (pmc or {}).get("_trace_forms"),
                     "issue": (dict(issue_bound(pmc, kern_s * 1e9), source=pmc_src) if pmc else None)},
        "build": build,
        "setup_s": round(setup_s, 2),
        "single_run_note": "one isolated search (enqueue -> complete, host turnaround included) on one handle, "
                           "median of 5 after the timed steps; ms_per_step is the pipelined throughput",
        "pipeline": (f"{nbuf} search handles on {'one stream' if args.one_stream else f'{nstr} streams'}: step i+{depth} "
                     f"enqueued before the host waits for step i (mp_search_enqueue/complete)"
                     if nbuf > 1 else "none: each step waits for the previous"),
        "scan_timing": ("HIP events around the scan kernel on its launch stream in every timed step"
                        if scan_in_timed else
                        "HIP events around the scan kernel on its launch stream in 3 untimed steps after the "
                        "timed ones, run one at a time (in the timed steps kernels of consecutive steps overlap)"),
    }
    if args.opts:
        out["search_options"] = args.opts
    if args.shard_of > 1:
        out["diagnostic"] = f"rank 0 of a {args.shard_of}-way owned-range split, alone on one GPU (not the metric)"
    if args.rehearse_one_gpu:
        out["diagnostic"] = f"{world} ranks sharing device 0 (rehearsal of the N-rank path, not the metric)"
    parity_ok = True
    if world > 1 or args.shard_of > 1:
        out["parity_distributed"] = dist_check
        parity_ok = dist_check["ok"]
    if world == 1 and not args.no_e2e:
        out["e2e"] = end_to_end(eng, table, names, lens, buf, offs, local, stream)
    if world == 1 and args.e2e_file:
        out["e2e_file"] = end_to_end_file(eng._sts_path, names, lens, buf, offs, cfg, local)
    if world == 1 and not args.no_cpu_baseline and args.shard_of <= 1:
        hits = search.fetch(nhits)
        threads = args.cpu_threads or host_cores()
        out["cpu_baseline"], otable, oprm = cpu_baseline(eng, lens, buf, offs, cfg, hits, args.cpu_budget, threads)
        parity_ok = out["cpu_baseline"]["parity_vs_gpu"]
        if not args.no_ref_model:
            out["cpu_baseline_reference_model"] = reference_model(otable, oprm, buf, offs, lens, threads,
                                                                  args.cpu_budget)
    print(json.dumps(out), flush=True)
    if world > 1:
        if comm is not None:
            comm.close()
        torch.distributed.destroy_process_group()
    if not parity_ok:
        log("FAIL: the GPU hit list differs from the CPU oracle's on the baseline sample")
        sys.exit(1)


if __name__ == "__main__":
    main()
