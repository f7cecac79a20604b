"""GPU parity: the HIP search path against the reference's golden outputs and the oracle.

Every case runs MerPCR.search / find_hits, i.e. the C-ABI library on the GPU,
and compares its output lines byte for byte with what the reference printed
(tests/golden/*.json.gz, produced by tests/golden/make_golden.py) or with the
CPU oracle (oracle/) on seeded synthetic inputs.
"""

import io
import os
import random
import tempfile

import numpy as np
import pytest

from merpcr_amd import FASTARecord, MerPCR, _native
from oracle import epcr_oracle as O
from tests.golden_io import data_path, load_golden

pytestmark = pytest.mark.gpu


def _engine(params):
    return MerPCR(**params)


def _load_sts(eng, text, td):
    p = os.path.join(td, "x.sts")
    with open(p, "w") as fh:
        fh.write(text)
    return eng.load_sts_file(p)


def _records(case, eng, td):
    if "fasta_text" in case:
        p = os.path.join(td, "x.fa")
        with open(p, "w", newline="") as fh:
            fh.write(case["fasta_text"])
        return eng.load_fasta_file(p)
    return [FASTARecord(defline=d, sequence=s) for d, s in case["records"]]


def _device_lines(eng, recs):
    hits = eng.find_hits(recs)
    return eng.format_hits(recs, hits)


def test_library_loaded_and_device_visible():
    from merpcr_amd import _native
    assert _native.device_count() >= 1


def test_search_then_torch_in_one_process():
    """A search before `import torch` leaves torch's device init working: the process
    maps one HIP runtime (_native._share_hip_runtime)."""
    import subprocess
    import sys
    code = ("import __graft_entry__ as g; g.smoke(); import torch; "
            "x = torch.ones(4, device='cuda:0'); assert float(x.sum()) == 4.0; "
            "maps = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}; "
            "assert len(maps) == 1, maps; print('one runtime', maps)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_bundled_kat():
    g = load_golden("bundled.json.gz")
    for case in g["cases"]:
        eng = _engine(case["params"])
        assert eng.load_sts_file(data_path("test.sts"))
        recs = eng.load_fasta_file(data_path("test.fa"))
        assert _device_lines(eng, recs) == case["output"].splitlines(), case["params"]


def test_bundled_search_to_file():
    eng = MerPCR(wordsize=11, mismatches=0, margin=50, threads=1)
    assert eng.load_sts_file(data_path("test.sts"))
    recs = eng.load_fasta_file(data_path("test.fa"))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "o.txt")
        n = eng.search(recs, out)
        text = open(out).read()
    assert n == 1 == eng.total_hits
    assert text == "L78833\t75823..76023\tAFM248yg9\t(D17S932)  Chr.17, 63.7 cM\t(-)\n"


@pytest.mark.parametrize("bits", [0, 1, 4, 5, 6, 7])
def test_dense_repeat_order(bits):
    """15,936 hits on an 8 kbp repeat; with 2 forced device-sort buckets they overflow the
    per-bucket capacity and the rocPRIM fallback orders them; with 16 buckets of ~1,000 keys
    some go to the crowded workgroup sort (over 1,024) and the rest to a wave's 1,024-slot
    register sort; 32, 64 and 128 buckets take the 1,024- and 256-slot register sorts."""
    case = load_golden("repeat.json.gz")
    eng = _engine(case["params"])
    eng.search_options = dict(sort_bucket_bits=bits)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, case["sts_text"], td)
        recs = _records(case, eng, td)
    lines = _device_lines(eng, recs)
    assert len(lines) == 15936
    assert lines == case["output"].splitlines()


@pytest.mark.parametrize("tails", ["auto", "inline", "kernel"])
@pytest.mark.parametrize("name", ["random_cases.json.gz", "special_cases.json.gz"])
def test_golden_corpus(name, tails):
    """Every recorded reference case through the default kernels (dense_kernel for W <= 9),
    and again through scan_kernel with the multi-record bucket tails forced to each of its
    two paths, with the two-pass 128-bit hit ordering and without deferring full-head
    buckets to tail_kernel (mp_search_options)."""
    opts = {}
    if tails != "auto":
        opts = dict(tails=tails, dense=False, sort="radix128", defer=False)
    cases = load_golden(name)["cases"]
    bad = []
    for i, case in enumerate(cases):
        eng = _engine(case["params"])
        eng.search_options = opts
        with tempfile.TemporaryDirectory() as td:
            ok = _load_sts(eng, case["sts_text"], td)
            assert ok == case["load_ok"], i
            if not ok:
                continue
            recs = _records(case, eng, td)
        lines = _device_lines(eng, recs)
        if lines != case["output"].splitlines():
            bad.append((i, case["params"], lines[:5], case["output"].splitlines()[:5]))
    assert not bad, bad[:3]


def test_key_group_tables_without_deferral():
    """Regression for the 16-B key references: an I = 0 key-group table that does
    not defer its full-head buckets runs a kRkf = 0 scan form, which writes 32-B references,
    so its tail pass must stay in the 32-B form.  The golden corpus holds such tables (one of
    them faulted when the choice followed the key groups alone); each gives the reference's
    lines, and the key-group tables that do defer are there too."""
    kinds = {"defer": 0, "no_defer": 0}
    bad = []
    for i, case in enumerate(load_golden("random_cases.json.gz")["cases"]):
        eng = _engine(case["params"])
        with tempfile.TemporaryDirectory() as td:
            if not _load_sts(eng, case["sts_text"], td):
                continue
            lay = eng.device_table().layout()
            if "kgrp" not in lay:
                continue
            recs = _records(case, eng, td)
        kinds["defer" if "defer_full" in lay else "no_defer"] += 1
        if _device_lines(eng, recs) != case["output"].splitlines():
            bad.append((i, case["params"], sorted(lay)))
    assert not bad, bad[:3]
    assert kinds["defer"] > 0 and kinds["no_defer"] > 0, kinds


@pytest.mark.parametrize("bits", [1, 4])
def test_device_sort_crowded_buckets(bits):
    """The device-count bucket sort with forced coarse buckets: 2 buckets overflow the
    per-bucket LDS capacity on the larger cases (rocPRIM fallback), 16 buckets rank
    hundreds of keys per workgroup.  Every golden case must still match byte for byte."""
    bad = []
    for name in ("special_cases.json.gz", "random_cases.json.gz"):
        for i, case in enumerate(load_golden(name)["cases"][:200]):
            eng = _engine(case["params"])
            eng.search_options = dict(sort_bucket_bits=bits)
            with tempfile.TemporaryDirectory() as td:
                if not _load_sts(eng, case["sts_text"], td):
                    continue
                recs = _records(case, eng, td)
            if _device_lines(eng, recs) != case["output"].splitlines():
                bad.append((name, i))
    assert not bad, bad[:5]


def _synthetic(seed, n_sts, glen, W, N, I, M=50, iupac_primers=False, nrun=False):
    rng = random.Random(seed)
    sts = []
    seq = [rng.choice("ACGT") for _ in range(glen)]
    if nrun:
        for _ in range(glen // 5000):
            a = rng.randrange(glen)
            seq[a:a + rng.randint(10, 400)] = ["N"] * min(400, glen - a)
            del seq[glen:]
    for s in range(n_sts):
        p1 = [rng.choice("ACGT") for _ in range(rng.randint(18, 25))]
        p2 = [rng.choice("ACGT") for _ in range(rng.randint(18, 25))]
        if iupac_primers:
            for p in (p1, p2):
                for _ in range(2):
                    p[rng.randrange(len(p) - 12)] = rng.choice("RYSWKMN")
        p1, p2 = "".join(p1), "".join(p2)
        size = rng.randint(100, 400)
        sts.append(f"S{s}\t{p1}\t{p2}\t{size}\talias{s}")
        if rng.random() < 0.8:
            amp = p2 + "".join(rng.choice("ACGT") for _ in range(size - len(p1) - len(p2) + rng.randint(-M, M)))
            amp += O.revcomp(p1)
            if N and rng.random() < 0.5:
                amp = list(amp)
                amp[rng.randrange(3, 10)] = rng.choice("ACGT")
                amp = "".join(amp)
            a = rng.randrange(max(1, glen - len(amp)))
            seq[a:a + len(amp)] = list(amp.lower() if rng.random() < 0.3 else amp)
            del seq[glen:]
    return "\n".join(sts) + "\n", "".join(seq)


@pytest.mark.parametrize("cfg", [
    dict(seed=1, n_sts=300, glen=300_000, W=11, N=0, I=0),
    dict(seed=2, n_sts=300, glen=300_000, W=11, N=1, I=0),
    dict(seed=3, n_sts=200, glen=200_000, W=8, N=2, I=1, iupac_primers=True),
    dict(seed=4, n_sts=200, glen=200_000, W=12, N=1, I=0, nrun=True),
    dict(seed=5, n_sts=100, glen=150_000, W=16, N=3, I=1, nrun=True),
])
def test_synthetic_vs_oracle(cfg):
    sts_text, seq = _synthetic(cfg["seed"], cfg["n_sts"], cfg["glen"], cfg["W"], cfg["N"], cfg["I"],
                               iupac_primers=cfg.get("iupac_primers", False), nrun=cfg.get("nrun", False))
    prm = dict(wordsize=cfg["W"], mismatches=cfg["N"], iupac_mode=cfg["I"], margin=50)
    eng = MerPCR(**prm)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    recs = [FASTARecord(defline=">chrS", sequence=seq)]
    got = _device_lines(eng, recs)
    table = O.load_sts_lines(sts_text.splitlines(True), cfg["W"], 240)
    exp = O.search_lines([("chrS", seq)], table, O.params(**prm))
    assert len(exp) > 0
    assert got == exp


def test_sharded_ranges_concatenate_to_whole():
    """Owned (seq, k) ranges partition the hit list exactly (multi-GPU invariant)."""
    from merpcr_amd import _native
    sts_text, seq = _synthetic(9, 200, 120_000, 10, 1, 0)
    eng = MerPCR(wordsize=10, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    seqs = [seq[:50_000], seq[50_000:50_500], "", seq[50_500:]]
    data = eng.encode_sequences(seqs)
    genome = _native.Genome(0, [len(d) for d in data])
    for i, d in enumerate(data):
        if len(d):
            genome.put(i, d)
    genome.seal()
    s = _native.Search(eng.device_table(), genome)
    whole = s.fetch(s.run())
    cuts = [(0, 0), (0, 17_001), (1, 100), (3, 0), (3, 33_333), (4, 0)]
    parts = []
    for (a, ka), (b, kb) in zip(cuts[:-1], cuts[1:]):
        parts.append(s.fetch(s.run((a, b, ka, kb))))
    cat = np.concatenate(parts)
    assert len(whole) > 0
    assert np.array_equal(cat, whole)


def test_chunk_emulation_matches_reference_threads():
    """-T N corpus: with emulate_chunks the GPU output equals the reference's
    multi-process output line for line (duplicates included); without it, every T
    gives the exact T=1 output."""
    for case in load_golden("chunked.json.gz")["cases"]:
        recs = [FASTARecord(defline=d, sequence=s) for d, s in case["records"]]
        t1 = case["by_threads"]["1"]["output"].splitlines()
        with tempfile.TemporaryDirectory() as td:
            for t, exp in case["by_threads"].items():
                eng = MerPCR(threads=int(t), emulate_chunks=True, **case["params"])
                assert _load_sts(eng, case["sts_text"], td)
                assert eng.max_pcr_size == case["max_pcr_size"]
                assert _device_lines(eng, recs) == exp["output"].splitlines(), (case["name"], t)
                eng.emulate_chunks = False
                assert _device_lines(eng, recs) == t1, (case["name"], t)


def test_cli_threads_emulation(tmp_path):
    """The CLI with -T 4 --emulate-chunks writes the reference's -T 4 output file."""
    from merpcr_amd.cli import main
    case = next(c for c in load_golden("chunked.json.gz")["cases"] if c["name"] == "seam")
    sts = tmp_path / "x.sts"
    sts.write_text(case["sts_text"])
    fa = tmp_path / "x.fa"
    fa.write_text("".join(f"{d}\n{s}\n" for d, s in case["records"]))
    out = tmp_path / "out.txt"
    p = case["params"]
    rc = main([str(sts), str(fa), "-W", str(p["wordsize"]), "-M", str(p["margin"]), "-N", str(p["mismatches"]),
               "-T", "4", "--emulate-chunks", "-O", str(out)])
    assert rc == 0
    assert out.read_text() == case["by_threads"]["4"]["output"]


@pytest.mark.parametrize("tails", ["auto", "inline", "kernel"])
@pytest.mark.parametrize("W,n_sts,glen,N,I,iupac", [(8, 4000, 3_000_000, 1, 0, 0.0), (9, 6000, 2_000_000, 2, 1, 0.1),
                                                    (11, 20000, 4_000_000, 1, 1, 0.1),
                                                    (11, 20000, 4_000_000, 2, 0, 0.1),  # 16-B heads, never bits
                                                    (12, 40000, 4_000_000, 1, 0, 0.0)])  # > 65536 keys: 2-bit LDS filter
def test_dense_tables_vs_c_oracle(tails, W, n_sts, glen, N, I, iupac):
    """Larger tables (multi-record buckets everywhere at W=8) through the default kernels
    and through scan_kernel with both tail paths, against the C oracle byte for byte, with
    planted amplicons and N runs."""
    from merpcr_amd import synth
    from oracle import c_oracle as C
    sts = synth.make_sts(n_sts, seed=7, W=W, iupac=iupac)
    rng = np.random.default_rng(3)
    g = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, glen)].copy()
    for _ in range(30):
        a = int(rng.integers(0, glen - 3000))
        g[a:a + int(rng.integers(50, 3000))] = ord("N")
    amps, starts = synth.amplicons(sts, glen, 7, N, 50, W)
    for amp, st in list(zip(amps, starts))[:: 3]:
        if st + len(amp) <= glen:
            g[st:st + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    seq = g.tobytes().decode("ascii")
    prm = dict(wordsize=W, mismatches=N, iupac_mode=I, margin=50)
    eng = MerPCR(**prm)
    if tails != "auto":
        eng.search_options = dict(tails=tails, dense=False)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts.text(), td)
    hits = eng.find_hits([FASTARecord(defline=">chrD", sequence=seq)])
    table = O.load_sts_lines(sts.text().splitlines(True), W, 240)
    ref = C.search(table, [g], O.params(**prm), 8)
    assert len(ref) > 100
    assert len(hits) == len(ref) and hits.tobytes() == ref.tobytes()


@pytest.mark.parametrize("W,I,N,X", [(6, 0, 1, 1), (7, 1, 2, 0), (8, 0, 0, 3), (8, 1, 1, 1), (9, 1, 1, 2)])
def test_dense_filter_edge_cases(W, I, N, X):
    """dense_kernel's filter and bucket index against the C oracle: keys shared by up to
    60 records (escape buckets walked through binfo), records the filter cannot carry
    (IUPAC bases after the seed, seed inside the primer, primers shorter than W + 7),
    genome IUPAC characters and U (passed straight to search), protected 3' bases."""
    from oracle import c_oracle as C
    rng = np.random.default_rng(100 + W * 10 + I)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)

    def rnd(n):
        return acgt[rng.integers(0, 4, n)].tobytes().decode()

    lines = []
    prefixes = [rnd(W) for _ in range(6)]
    for i in range(900):
        l1, l2 = int(rng.integers(18, 26)), int(rng.integers(18, 26))
        p1, p2 = rnd(l1), rnd(l2)
        kind = i % 9
        if kind in (0, 1):                 # shared seed keys: large buckets
            p1 = prefixes[i % 6] + p1[W:]
        elif kind == 2:                    # IUPAC base after the seed
            j = W + int(rng.integers(0, 7))
            p1 = p1[:j] + "RYKMSWN"[i % 7] + p1[j + 1:]
        elif kind == 3:                    # seed inside the primer
            p1 = "N" + p1[1:]
        elif kind == 4:                    # too short to carry the filter
            p1 = p1[:W + int(rng.integers(0, 5))]
        lines.append(f"S{i}\t{p1}\t{p2}\t{int(rng.integers(80, 300))}\n")
    sts_text = "".join(lines)
    table = O.load_sts_lines(sts_text.splitlines(True), W, 240)
    glen = 600_000
    g = acgt[rng.integers(0, 4, glen)].copy()
    # plant amplicons of the STS (both orientations), some with a mismatch
    for i in range(0, 900, 2):
        _, p1, p2, size = lines[i].rstrip("\n").split("\t")[:4]
        a = p1.replace("N", "A")
        b = O.revcomp(p1)
        for x, y in ((a, p2), (p2, b)):
            x = "".join(c if c in "ACGT" else "G" for c in x)
            y = "".join(c if c in "ACGT" else "C" for c in y)
            amp = (x + rnd(max(int(size) - len(x) - len(y), 0)) + y).encode()
            st = int(rng.integers(0, glen - len(amp)))
            g[st:st + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    # genome IUPAC characters and U
    for c, frac in ((b"N", 0.004), (b"R", 0.002), (b"Y", 0.002), (b"W", 0.001), (b"U", 0.002)):
        idx = rng.integers(0, glen, int(glen * frac))
        g[idx] = c[0]
    prm = dict(wordsize=W, mismatches=N, iupac_mode=I, margin=50, three_prime_match=X)
    eng = MerPCR(**prm)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    seq = g.tobytes().decode("ascii")
    hits = eng.find_hits([FASTARecord(defline=">chrE", sequence=seq)])
    ref = C.search(table, [g], O.params(**prm), 8)
    assert len(ref) > 50
    assert len(hits) == len(ref) and hits.tobytes() == ref.tobytes()


@pytest.mark.parametrize("W", [11, 12])
def test_seed_queue_rounds(W):
    """Every window a seed (a periodic genome whose 11/12-mers are all keys): the scan
    kernel's per-wave seed queue overflows and drains in rounds; against the C oracle."""
    from oracle import c_oracle as C
    rng = np.random.default_rng(W)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    unit = acgt[rng.integers(0, 4, 97)].tobytes().decode()
    g = (unit * 260)[:25_000]
    lines = []
    for i in range(97):
        s = (unit * 3)[i:]
        p1, p2 = s[:20], s[150:170]
        lines.append(f"P{i}\t{p1}\t{p2}\t{150 + 20 + int(rng.integers(-3, 4))}\n")
    sts_text = "".join(lines)
    prm = dict(wordsize=W, mismatches=1, margin=5)
    eng = MerPCR(**prm)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    hits = eng.find_hits([FASTARecord(defline=">chrP", sequence=g)])
    table = O.load_sts_lines(sts_text.splitlines(True), W, 240)
    ref = C.search(table, [np.frombuffer(g.encode(), dtype=np.uint8)], O.params(**prm), 8)
    assert len(ref) > 1000
    assert len(hits) == len(ref) and hits.tobytes() == ref.tobytes()


@pytest.mark.parametrize("N,X", [(0, 0), (1, 1), (2, 0)])
def test_full_head_prefilter_buckets(N, X):
    """Buckets of 2-4 records that share a primer-1 seed (kHead8Filt prefilter on the full
    8-B head for 1-3 records, plain deferral for 4), some also sharing the filter bases,
    with planted amplicons of every record: the deferring drain against the C oracle."""
    from merpcr_amd import synth
    from oracle import c_oracle as C
    W = 11
    sts = synth.make_sts(6000, seed=11, W=W)
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    # ~1.5% of the buckets shared, so the drain defers full heads (under 5% of them)
    for i in range(0, 450, 3):  # groups: record i's first W (or W + 4) bases copied to i+1, i+2
        for j in (1, 2):
            keep = W + (4 if rng.random() < 0.3 else 0)
            tail = acgt[rng.integers(0, 4, len(sts.p1[i + j]) - keep)].tobytes()
            sts.p1[i + j] = sts.p1[i][:keep] + tail
    for i in range(3000, 3040, 4):  # a few 4-record buckets
        for j in (1, 2, 3):
            sts.p1[i + j] = sts.p1[i][:W] + sts.p1[i + j][W:]
    glen = 5_000_000
    g = acgt[rng.integers(0, 4, glen)].copy()
    amps, starts = synth.amplicons(sts, glen, 13, N, 50, W)
    for amp, st in zip(amps, starts):
        if st + len(amp) <= glen:
            g[st:st + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    seq = g.tobytes().decode("ascii")
    prm = dict(wordsize=W, mismatches=N, three_prime_match=X, margin=50)
    eng = MerPCR(**prm)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts.text(), td)
    hits = eng.find_hits([FASTARecord(defline=">chrH", sequence=seq)])
    table = O.load_sts_lines(sts.text().splitlines(True), W, 240)
    ref = C.search(table, [g], O.params(**prm), 8)
    assert len(ref) > 1000
    assert len(hits) == len(ref) and hits.tobytes() == ref.tobytes()


def test_forced_regrowth_is_identical():
    """Survivor, bucket-tail and hit lists created one entry long (mp_search_options):
    every list overflows, is regrown and its producers rerun; the output is byte-identical
    to the default capacities and the regrowths are counted."""
    sts_text, seq = _synthetic(21, 300, 300_000, 11, 1, 0)
    recs = [FASTARecord(defline=">chrG", sequence=seq)]
    ref_eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(ref_eng, sts_text, td)
    exp = _device_lines(ref_eng, recs)
    for opts in (dict(hit_cap=1, surv_cap=1, tail_cap=1), dict(hit_cap=1),
                 dict(hit_cap=1, surv_cap=1, tail_cap=1, tails="inline", dense=False)):
        eng = MerPCR(wordsize=11, mismatches=1)
        eng.search_options = opts
        with tempfile.TemporaryDirectory() as td:
            assert _load_sts(eng, sts_text, td)
        assert _device_lines(eng, recs) == exp, opts
        assert eng.last_search_stats["regrowths"] >= 1, opts
    assert len(exp) > 100


def test_pending_run_guards():
    """Between mp_search_enqueue and mp_search_complete the run owns the handle's lists:
    fetch, stats and the genome's writers fail with MP_E_STATE instead of reading a list
    being written; complete then returns the same hits; destroying a handle with a run
    still enqueued waits for it."""
    sts_text, seq = _synthetic(23, 200, 300_000, 11, 1, 0)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    g = _native.Genome(0, [len(seq)])
    g.put(0, seq.encode())
    g.seal()
    s = _native.Search(eng.device_table(), g)
    n = s.run()
    ref = s.fetch(n)
    assert n > 10
    s.enqueue()
    for fn in (lambda: s.fetch(n), s.last_stats, s.device_hits, lambda: g.reset([len(seq)]),
               lambda: g.put(0, b"ACGT")):
        with pytest.raises(_native.NativeError) as ei:
            fn()
        assert ei.value.code == _native.MP_E_STATE, ei.value
    n2 = s.complete()
    assert n2 == n and s.fetch(n2).tobytes() == ref.tobytes()
    assert s.dev_bytes() > 0
    s.enqueue()
    s.close()  # waits for the enqueued run
    g.reset([len(seq)])  # no run pending any more
    g.close()


def test_handles_reused_across_searches():
    """One engine, several search() calls of different sizes and record counts: the genome
    and search handles are re-laid out (mp_genome_reset), the results equal a fresh engine's;
    a repeated small search orders its hits in well under a millisecond."""
    sts_text, seq = _synthetic(22, 200, 400_000, 11, 1, 0, nrun=True)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    sets = [[seq], [seq[:50_000], seq[50_000:51_000]], [seq[100_000:]], ["ACGT" * 5, "", seq[:200_000]], [seq]]
    for seqs in sets:
        recs = [FASTARecord(defline=f">r{i}", sequence=s) for i, s in enumerate(seqs)]
        fresh = MerPCR(wordsize=11, mismatches=1)
        with tempfile.TemporaryDirectory() as td:
            assert _load_sts(fresh, sts_text, td)
        assert _device_lines(eng, recs) == _device_lines(fresh, recs)
    small = [FASTARecord(defline=">s", sequence=seq[:120_000])]
    eng.find_hits(small)
    eng.find_hits(small)
    assert eng.last_search_stats["order_ms"] < 1.0, eng.last_search_stats


def test_latin1_primer_character_first_search():
    """A Latin-1 primer character ('É', not IUPAC: literal equality) matched by the same
    genome character: the first search after load_sts_file already finds the hit (its byte
    code is registered before the genome is encoded), and repeated searches agree."""
    p1, p2 = "ACGTTGCAAGCTTAGCÉA", "GGATCCTTAGGCATCAGG"
    body = "".join(random.Random(5).choice("ACGT") for _ in range(400))
    seq = body[:100] + p1 + body[100:250] + p2 + body[250:]  # the "+" record: p1 ... p2 literal
    sts_text = f"LAT\t{p1}\t{p2}\t{len(p1) + 150 + len(p2)}\n"
    prm = dict(wordsize=8, mismatches=0, margin=5)
    eng = MerPCR(**prm)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    recs = [FASTARecord(defline=">lat", sequence=seq)]
    table = O.load_sts_lines(sts_text.splitlines(True), 8, 240)
    exp = O.search_lines([("lat", seq)], table, O.params(**prm))
    assert len(exp) == 1
    assert _device_lines(eng, recs) == exp
    assert _device_lines(eng, recs) == exp


def _multi_case(W, n_sts, seed):
    """A multi-record synthetic genome (N runs, planted amplicons) and its STS text."""
    from merpcr_amd import synth
    sts = synth.make_sts(n_sts, seed=seed, W=W)
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    glen = 2_000_000
    g = acgt[rng.integers(0, 4, glen)].copy()
    for _ in range(20):
        a = int(rng.integers(0, glen - 3000))
        g[a:a + int(rng.integers(50, 3000))] = ord("N")
    amps, starts = synth.amplicons(sts, glen, seed, 1, 50, W)
    for amp, st in zip(amps, starts):
        if st + len(amp) <= glen:
            g[st:st + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    s = g.tobytes().decode("ascii")
    seqs = [s[:700_001], s[700_001:700_300], "", s[700_300:1_500_000], s[1_500_000:]]
    return sts.text(), seqs


@pytest.mark.parametrize("W,n_sts,opts", [(8, 3000, {}), (10, 3000, {}), (11, 6000, {}),
                                          (11, 6000, dict(tails="inline")), (11, 6000, dict(defer=False)),
                                          (12, 6000, {}), (11, 6000, dict(scan_grid=37)),
                                          (11, 6000, dict(ref32=True)), (8, 3000, dict(ref32=True))])
def test_sharded_ranges_all_paths(W, n_sts, opts):
    """Owned (seq, k) ranges partition the hit list exactly through every scan path:
    dense_kernel or the split seeds (W=8), the exact-LDS scan (W=10), the key-group scan with
    its references to tail_kernel (W=11 default; 16-B and, with ref32, 32-B references),
    inline tails, no deferral; cuts inside super-steps and next to records' seed offsets
    (k + hash_offset straddling a cut)."""
    from merpcr_amd import _native
    sts_text, seqs = _multi_case(W, n_sts, 30 + W)
    eng = MerPCR(wordsize=W, mismatches=1)
    eng.search_options = opts
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    data = eng.encode_sequences(seqs)
    genome = _native.Genome(0, [len(d) for d in data])
    for i, d in enumerate(data):
        if len(d):
            genome.put(i, d)
    genome.seal()
    s = _native.Search(eng.device_table(), genome)
    if opts:
        s.set_options(**opts)
    whole = s.fetch(s.run())
    assert len(whole) > 100
    # a grid of 37 scan workgroups (uneven XCD groups), or the key-group scans' references in the
    # 32-B form (the default is 16-B since round 6): the default handle's list
    if "scan_grid" in opts or "ref32" in opts:
        d = _native.Search(eng.device_table(), genome)
        assert np.array_equal(d.fetch(d.run()), whole)
        d.close()
    # cuts: mid super-step, at a hit's k, one and W-1 bases after a hit's k (its seed window
    # lies across the cut), record boundaries
    k0 = int(whole["pos1"][len(whole) // 3])
    q0 = int(whole["seq"][len(whole) // 3])
    k1 = int(whole["pos1"][2 * len(whole) // 3])
    q1 = int(whole["seq"][2 * len(whole) // 3])
    cuts = sorted({(0, 0), (0, 17_001), (q0, k0), (q0, k0 + 1), (q1, k1 + W - 1), (1, 100), (3, 0),
                   (3, 333_333), (len(seqs), 0)})
    parts = [s.fetch(s.run((a, b, ka, kb))) for (a, ka), (b, kb) in zip(cuts[:-1], cuts[1:])]
    cat = np.concatenate(parts)
    assert np.array_equal(cat, whole)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0]])
def test_multi_device_engine_matches_single(devices):
    """MerPCR(devices=[...]) / CLI --gpus: owned ranges over the devices, each packing only
    its share of the genome, gathered into devices[0] by the copy engines (hipMemcpyPeerAsync
    on devices[0]'s stream); identical to one device.  A repeated device (one GPU here) takes
    the same gather code as distinct devices do (mp_multi_run has one copy path)."""
    sts_text, seqs = _multi_case(11, 6000, 41)
    recs = [FASTARecord(defline=f">m{i}", sequence=s) for i, s in enumerate(seqs)]
    single = MerPCR(wordsize=11, mismatches=1)
    multi = MerPCR(wordsize=11, mismatches=1, devices=devices)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(single, sts_text, td)
        assert _load_sts(multi, sts_text, td)
    exp = _device_lines(single, recs)
    assert len(exp) > 100
    assert _device_lines(multi, recs) == exp
    assert _device_lines(multi, recs[1:]) == _device_lines(single, recs[1:])  # re-laid out, same handles
    assert len(multi.last_search_stats["devices"]) == len(devices)


def test_multi_rccl_gather_one_device():
    """mp_multi over one device with the gather switched to RCCL (mp_multi_set_gather:
    ncclCommInitAll, grouped ncclSend/ncclRecv to itself) gathers the hit list; a repeated
    device refuses it (RCCL admits one rank per device)."""
    from merpcr_amd import _native
    sts_text, seqs = _multi_case(11, 3000, 43)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    data = eng.encode_sequences(seqs)
    exp = eng.find_hits([FASTARecord(defline=f">m{i}", sequence=s) for i, s in enumerate(seqs)])
    m = _native.Multi([0], [eng.device_table()])
    m.set_gather("rccl")
    m.genome([len(d) for d in data])
    for i, d in enumerate(data):
        if len(d):
            m.put(i, d)
    m.seal()
    got = m.fetch(m.run())
    assert len(exp) > 100 and got.tobytes() == exp.tobytes()
    m.close()
    rep = _native.Multi([0, 0], [eng.device_table(), eng.device_table()])
    with pytest.raises(ValueError):
        rep.set_gather("rccl")
    rep.close()


def test_comm_gather_single_rank():
    """mp_comm_* with one rank: unique id -> communicator -> gather into a device buffer."""
    import torch
    from merpcr_amd import _native
    sts_text, seqs = _multi_case(10, 3000, 44)
    eng = MerPCR(wordsize=10, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    exp = eng.find_hits([FASTARecord(defline=f">m{i}", sequence=s) for i, s in enumerate(seqs)])
    comm = _native.Comm(_native.comm_unique_id(), 1, 0, 0)
    out = torch.empty(len(exp) * 24 + 24, dtype=torch.uint8, device="cuda:0")
    search = eng._dev_search
    n = comm.gather_hits(search, out.data_ptr(), len(exp) + 1, seq_shift=3)
    torch.cuda.synchronize()
    got = np.frombuffer(out[:n * 24].cpu().numpy().tobytes(), dtype=exp.dtype)
    assert n == len(exp) and np.array_equal(got["seq"], exp["seq"] + 3)
    assert np.array_equal(got["pos1"], exp["pos1"]) and np.array_equal(got["rec"], exp["rec"])
    with pytest.raises(_native.NativeError):  # rank 0's buffer too small: MP_E_CAP, nothing sent
        comm.gather_hits(search, out.data_ptr(), 1)
    assert comm.last_total == len(exp)
    comm.close()


def _two_rank_worker(rank, world, port, sts_text, seqs, q):
    import torch
    import torch.distributed as dist
    from merpcr_amd import _native
    from merpcr_amd.dist import as_hits, gather_hits, shard_ranges
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    data = eng.encode_sequences(seqs)
    genome = _native.Genome(0, [len(d) for d in data])
    for i, d in enumerate(data):
        if len(d):
            genome.put(i, d)
    genome.seal()
    s = _native.Search(eng.device_table(), genome)
    rng = shard_ranges([len(d) for d in data], world)[rank]
    mine = s.fetch(s.run(rng))  # the HIP path on this rank's owned range
    buf = torch.from_numpy(np.frombuffer(mine.tobytes() + b"\0" * 24, dtype=np.uint8).copy())
    got = gather_hits(buf, len(mine))
    if rank == 0:
        q.put(as_hits(got).tobytes())
    dist.barrier()
    dist.destroy_process_group()


def _two_rank_ipc_worker(rank, world, port, sts_text, seqs, q, steps, cap0=0):
    """One rank of the copy-engine gather (merpcr_amd.dist.IpcGather): `steps` runs of its
    owned range on two pipelined handles, each put into rank 0's region slot of its handle on
    the run's stream, as bench.py does.  cap0 > 0: regions of cap0 hits, too small, so every
    put fails with MP_E_CAP and settle() must regrow them."""
    import torch
    import torch.distributed as dist
    from merpcr_amd import _native
    from merpcr_amd.dist import IpcGather, shard_ranges
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    data = eng.encode_sequences(seqs)
    genome = _native.Genome(0, [len(d) for d in data])
    for i, d in enumerate(data):
        if len(d):
            genome.put(i, d)
    genome.seal()
    hs = [_native.Search(eng.device_table(), genome) for _ in range(2)]
    rng = shard_ranges([len(d) for d in data], world)[rank]
    n = hs[0].run(rng)
    g = IpcGather(0, cap0 or max(64, 2 * n), slots=2)
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    fits = []
    for i in range(steps):
        j = i % 2
        hs[j].enqueue(rng, sts[j].cuda_stream)
        hs[j].complete()
        fits.append(g.put(hs[j], sts[j].cuda_stream, slot=j))
    torch.cuda.synchronize()
    dist.barrier()
    grown = g.settle()
    last = (steps - 1) % 2
    if rank == 0:
        q.put((g.counts(last), g.hits(slot=last).cpu().numpy().tobytes(), grown, fits, g.cap))
    g.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cap0", [0, 8])
def test_two_ranks_ipc_gather_on_one_gpu(cap0):
    """bench.py's default N > 1 gather (copy-engine puts into rank 0's regions, mapped by IPC
    in the other process): two processes on cuda:0, three steps each on two pipelined handles
    with a region slot each; rank 0's rank-ordered regions equal the whole-genome HIP list and
    the C oracle's.  cap0 = 8: every put overflows (MP_E_CAP, nothing copied) and the
    collective settle() regrows the regions and puts each slot's last run again."""
    import socket
    import torch.multiprocessing as tmp
    from oracle import c_oracle as C
    sts_text, seqs = _multi_case(11, 3000, 45)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_ipc_worker, args=(r, 2, port, sts_text, seqs, q, 3, cap0)) for r in range(2)]
    for p in procs:
        p.start()
    counts, got, grown, fits, cap = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    whole = eng.find_hits([FASTARecord(defline=f">m{i}", sequence=x) for i, x in enumerate(seqs)])
    table = O.load_sts_lines(sts_text.splitlines(True), 11, 240)
    ref = C.search(table, [np.frombuffer(x.encode(), dtype=np.uint8) for x in seqs], O.params(wordsize=11, mismatches=1), 8)
    assert len(whole) > 100 and sum(counts) == len(whole) and min(counts) > 0
    assert got == whole.tobytes() == ref.tobytes()
    assert all(p.exitcode == 0 for p in procs)
    if cap0:
        assert grown and not any(fits) and cap >= max(counts), (grown, fits, cap, counts)
    else:
        assert not grown and all(fits)


def test_two_ranks_on_one_gpu():
    """Two processes on cuda:0, each searching its owned range with the HIP path, gathered
    over torch.distributed (gloo: RCCL does not admit two ranks on one GPU); the gathered
    list equals the whole-genome HIP list and the C oracle's."""
    import socket
    import torch.multiprocessing as tmp
    from oracle import c_oracle as C
    sts_text, seqs = _multi_case(11, 3000, 45)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, sts_text, seqs, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    eng = MerPCR(wordsize=11, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    whole = eng.find_hits([FASTARecord(defline=f">m{i}", sequence=x) for i, x in enumerate(seqs)])
    table = O.load_sts_lines(sts_text.splitlines(True), 11, 240)
    ref = C.search(table, [np.frombuffer(x.encode(), dtype=np.uint8) for x in seqs], O.params(wordsize=11, mismatches=1), 8)
    assert len(whole) > 100 and got == whole.tobytes() == ref.tobytes()
    assert all(p.exitcode == 0 for p in procs)


def test_iupac_wide_key_groups_with_genome_ambiguity():
    """I = 1 tables whose primers carry IUPAC bases right after the seed (c4's shape) take
    the wide key groups (kgrp4: ten bases per field, kgrp_pass4).  Genome IUPAC characters
    inside those bases match under I = 1 although the 2-bit plane reads them as 'A': such
    windows must pass on presence alone.  Planted amplicons put N/R/Y/K into exactly those
    positions."""
    rng = random.Random(41)
    W, N, M, glen = 11, 2, 50, 250_000
    seq = [rng.choice("ACGT") for _ in range(glen)]
    sts = []
    for s in range(300):
        p1 = [rng.choice("ACGT") for _ in range(rng.randint(20, 25))]
        p2 = [rng.choice("ACGT") for _ in range(rng.randint(20, 25))]
        for p in (p1, p2):  # IUPAC bases among primer bases W..W+12, none in the seed
            for _ in range(2):
                p[rng.randrange(W, min(len(p) - 3, W + 13))] = rng.choice("RYSWKMN")
        p1, p2 = "".join(p1), "".join(p2)
        size = rng.randint(120, 400)
        sts.append(f"W{s}\t{p1}\t{p2}\t{size}\tw{s}")
        for form in (0, 1):
            a_, b_ = (p1, p2) if form == 0 else (p2, O.revcomp(p1))
            a_ = list(a_.replace("R", "A").replace("Y", "C").replace("S", "G").replace("W", "T")
                      .replace("K", "G").replace("M", "C").replace("N", "T"))
            for _ in range(rng.randint(0, 2)):  # genome ambiguity characters after the seed
                a_[rng.randrange(W, min(len(a_), W + 13))] = rng.choice("NRYK")
            fill = "".join(rng.choice("ACGT") for _ in range(max(0, size - len(a_) - len(b_) + rng.randint(-M, M))))
            amp = "".join(a_) + fill + b_
            at = rng.randrange(glen - len(amp))
            seq[at:at + len(amp)] = list(amp)
    for _ in range(40):  # N runs
        at = rng.randrange(glen - 200)
        seq[at:at + rng.randint(1, 150)] = "N" * 150
    seq = "".join(seq)[:glen]
    sts_text = "\n".join(sts) + "\n"
    prm = dict(wordsize=W, mismatches=N, iupac_mode=1, margin=M)
    eng = MerPCR(**prm)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    recs = [FASTARecord(defline=">chrW", sequence=seq)]
    got = _device_lines(eng, recs)
    table = O.load_sts_lines(sts_text.splitlines(True), W, 240)
    exp = O.search_lines([("chrW", seq)], table, O.params(**prm))
    assert len(exp) > 200
    assert got == exp


@pytest.mark.parametrize("W,N,iupac,n_sts", [(11, 2, 0.1, 30000), (11, 2, 0.1, 100000), (11, 1, 0.3, 30000),
                                             (12, 2, 0.1, 40000), (13, 2, 0.1, 40000), (13, 2, 0.2, 40000)])
def test_wide_key_groups_vs_rank_heads(W, N, iupac, n_sts):
    """The I = 1 scan through the wide key groups (kgrp4, the default for c4-shaped tables)
    and through the rank words and 8-B IUPAC heads (table option kgrp4="never") give the C
    oracle's hit list byte for byte: primers with IUPAC bases after the
    seed, short primers (fields past the primer's end), multi-record keys, groups with more
    than three present keys, N runs and planted amplicons.  kgrp4="always" builds the wide key
    groups whenever the table can carry them (the pass-rate estimate skipped); a table that
    takes the I = 1 8-B fields instead (kgrp_wild) is checked on that path in both runs.
    100k STS at W = 11 (c4's table): ~6% of the groups hold four or more keys and ~2% of the
    keys have two records."""
    from merpcr_amd import synth
    from oracle import c_oracle as C
    sts = synth.make_sts(n_sts, seed=11 + W, W=W, iupac=iupac)
    rng = np.random.default_rng(W)
    glen = 3_000_000
    g = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, glen)].copy()
    for _ in range(20):
        a = int(rng.integers(0, glen - 3000))
        g[a:a + int(rng.integers(50, 3000))] = ord("N")
    amps, starts = synth.amplicons(sts, glen, 5, N, 50, W)
    step = max(2, -(-460 // (glen // len(amps))))  # every step-th slot: planted amplicons do not overlap
    for amp, st in list(zip(amps, starts))[::step]:
        if st + len(amp) <= glen:
            g[st:st + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    seq = g.tobytes().decode("ascii")
    prm = dict(wordsize=W, mismatches=N, iupac_mode=1, margin=50)
    table = O.load_sts_lines(sts.text().splitlines(True), W, 240)
    ref = C.search(table, [g], O.params(**prm), 8)
    assert len(ref) > 100
    lays = []
    for no4 in ("always", "never"):
        eng = MerPCR(**prm)
        eng.table_options = {"kgrp4": no4}
        with tempfile.TemporaryDirectory() as td:
            assert _load_sts(eng, sts.text(), td)
        hits = eng.find_hits([FASTARecord(defline=">chrK", sequence=seq)])
        assert len(hits) == len(ref) and hits.tobytes() == ref.tobytes(), no4
        lays.append(eng.device_table().layout())
    # the two runs took different level-2 structures (else the A/B compares a path with itself),
    # unless the table is a kgrp_wild one, which never carries the wide groups
    assert "kgrp4" not in lays[1]
    assert "kgrp4" in lays[0] or "kgrp" in lays[0], lays
    if (W, N) == (11, 2):  # c4's shape: the wide groups must be what the first run took
        assert "kgrp4" in lays[0], lays


def test_primer_edit_in_place_vs_oracle():
    """A primer edited in place after load: the reference still finds the record through the
    bucket of its load-time key (engine.py:265-279, 483-486) and compares the primer it holds
    now (engine.py:507-597).  Two edits: one after the seed (the edited primer is found), one
    inside the seed (the genome carries the new primer, whose first W-mer is not the key, so
    neither engine may report it)."""
    rng = random.Random(7)
    W = 11

    def rnd(n):
        return "".join(rng.choice("ACGT") for _ in range(n))

    a1, a2, b1, b2 = rnd(22), rnd(21), rnd(20), rnd(23)
    a1_new = a1[:15] + ("A" if a1[15] != "A" else "C") + a1[16:]      # edit past the seed
    b1_new = ("G" if b1[0] != "G" else "T") + b1[1:]                   # edit inside the seed
    sts_text = f"A\t{a1}\t{a2}\t200\talias A\nB\t{b1}\t{b2}\t180\n"
    fill_a = rnd(200 - len(a1) - len(a2))
    fill_b = rnd(180 - len(b1) - len(b2))
    genome = rnd(5000) + a1_new + fill_a + a2 + rnd(3000) + b1_new + fill_b + b2 + rnd(4000)
    params = dict(wordsize=W, mismatches=0, margin=50)
    eng = MerPCR(**params)
    with tempfile.TemporaryDirectory() as td:
        assert _load_sts(eng, sts_text, td)
    recs = [FASTARecord(defline=">g1 test", sequence=genome)]
    assert _device_lines(eng, recs) == []                # neither primer as loaded is in the genome
    plus = [r for r in eng.sts_records if r.direct == "+"]
    plus[0].primer1 = a1_new
    plus[1].primer1 = b1_new
    got = _device_lines(eng, recs)
    table = O.load_sts_lines(sts_text.splitlines(True), W, 240)
    orec = [r for r in table.records if r.direct == "+"]
    orec[0].primer1 = a1_new                            # same edit, key left as loaded
    orec[1].primer1 = b1_new
    exp = O.search_lines([("g1", genome)], table, O.params(**params))
    assert got == exp
    assert len(exp) == 1 and exp[0].split("\t")[2] == "A", exp
