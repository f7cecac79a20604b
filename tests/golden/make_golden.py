"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run only in the build container, where the reference is importable:

    PYTHONPATH=/root/reference/src python3 tests/golden/make_golden.py
    PYTHONPATH=/root/reference/src python3 tests/golden/make_golden.py --chunked   # -T N corpus
    PYTHONPATH=/root/reference/src python3 tests/golden/make_golden.py --errors    # error paths

The reference never ships with this repository and never runs on the GPU box;
what is committed is data only: the seeded inputs each case was built from and
the exact output the reference printed for them (plus unit-level known-answer
vectors for its helper functions).  The case generator below is this build's
own code.
"""

from __future__ import annotations

import gzip
import hashlib
import io
import json
import logging
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "data")

IUPAC_EXTRA = "RYMKSWBDHVN"


def _ref():
    from merpcr import MerPCR  # noqa: F401  (reference, build container only)
    from merpcr.core.models import FASTARecord
    return MerPCR, FASTARecord


# --------------------------------------------------------------------------
# seeded case generator (this build's own code)
# --------------------------------------------------------------------------

def _rc(s):
    comp = {"A": "T", "C": "G", "G": "C", "T": "A", "U": "A", "B": "V", "V": "B",
            "D": "H", "H": "D", "K": "M", "M": "K", "R": "Y", "Y": "R",
            "N": "N", "S": "S", "W": "W", "X": "X"}
    return "".join(comp.get(c.upper(), "N") for c in reversed(s))


def _rand_seq(rng, n, mode):
    if n <= 0:
        return ""
    if mode == "acgt":
        return "".join(rng.choice("ACGT") for _ in range(n))
    if mode == "lowcomplex":
        alpha = rng.choice(["AT", "GC", "AC", "ACG", "A"])
        return "".join(rng.choice(alpha) for _ in range(n))
    if mode == "nruns":
        out = []
        while len(out) < n:
            if rng.random() < 0.08:
                out.extend("N" * rng.randint(1, 40))
            else:
                out.extend(rng.choice("ACGT") for _ in range(rng.randint(5, 120)))
        return "".join(out[:n])
    if mode == "iupac":
        return "".join(rng.choice("ACGT" * 6 + IUPAC_EXTRA + "X") for _ in range(n))
    if mode == "mixedcase":
        return "".join(rng.choice("ACGTacgt") for _ in range(n))
    if mode == "rna":
        return "".join(rng.choice("ACGU" + "ACGT" * 3) for _ in range(n))
    if mode == "junk":
        return "".join(rng.choice("ACGT" * 8 + "Nn*-.Z0x ") for _ in range(n))
    raise ValueError(mode)


def _mutate(rng, s, k, protect_tail=0, protect_head=0):
    s = list(s)
    L = len(s)
    for _ in range(k):
        lo = protect_head
        hi = L - 1 - protect_tail
        if hi < lo:
            break
        i = rng.randint(lo, hi)
        s[i] = rng.choice([c for c in "ACGT" if c != s[i].upper()] or ["A"])
    return "".join(s)


def _primer(rng, L, style):
    if style == "acgt":
        return "".join(rng.choice("ACGT") for _ in range(L))
    if style == "lower":
        return "".join(rng.choice("ACGTacgt") for _ in range(L))
    if style == "iupac":
        p = [rng.choice("ACGT") for _ in range(L)]
        for _ in range(rng.randint(1, max(1, L // 5))):
            p[rng.randrange(L)] = rng.choice(IUPAC_EXTRA)
        return "".join(p)
    if style == "rna":
        return "".join(rng.choice("ACGU") for _ in range(L))
    if style == "weird":
        p = [rng.choice("ACGT") for _ in range(L)]
        for _ in range(rng.randint(1, 3)):
            p[rng.randrange(L)] = rng.choice("XZ-*nr")
        return "".join(p)
    raise ValueError(style)


def _size_field(rng, size):
    r = rng.random()
    if r < 0.65:
        return str(size)
    if r < 0.8:
        a = max(1, size - rng.randint(0, 30))
        return f"{a}-{2 * size - a}"
    return rng.choice(["-5", "0", "abc", "10-", "-", "1-2-3", "x-y", " 7", "150", "3"])


def gen_case(rng, idx):
    W = rng.choice([3, 4, 5, 6, 7, 8, 8, 9, 10, 11, 11, 11, 12, 13, 14, 16])
    M = rng.choice([0, 1, 3, 10, 50, 50])
    N = rng.choice([0, 0, 1, 1, 2, 3])
    X = rng.choice([0, 1, 1, 2, 4, 40])
    I = rng.choice([0, 0, 1])
    Z = rng.choice([240, 240, 100, 60])
    mode = rng.choice(["acgt", "acgt", "acgt", "nruns", "iupac", "mixedcase",
                       "lowcomplex", "rna", "junk"])
    n_sts = rng.randint(1, 10)
    sts_lines = []
    planted = []
    for s in range(n_sts):
        L1 = rng.randint(W, max(W, 26))
        L2 = rng.randint(W, max(W, 26))
        style = rng.choice(["acgt"] * 6 + ["lower", "iupac", "rna", "weird"])
        p1 = _primer(rng, L1, style)
        p2 = _primer(rng, L2, rng.choice(["acgt", "acgt", style]))
        size = rng.randint(max(1, L1 + L2 - 10), L1 + L2 + 250)
        field = _size_field(rng, size)
        alias = rng.choice(["", "alias%d" % s, "(D17S%d)  Chr.1, 2.0 cM" % s])
        cols = [f"STS{idx}_{s}", p1, p2, field]
        if alias or rng.random() < 0.3:
            cols.append(alias)
        if rng.random() < 0.05:
            cols.append("extra")
        sts_lines.append("\t".join(cols))
        if rng.random() < 0.08:
            sts_lines.append(sts_lines[-1])  # duplicate line -> duplicate hits
        planted.append((p1, p2, size))
    if rng.random() < 0.2:
        sts_lines.insert(rng.randrange(len(sts_lines) + 1), "# comment line")
    if rng.random() < 0.15:
        sts_lines.insert(rng.randrange(len(sts_lines) + 1), "")
    if rng.random() < 0.02:
        sts_lines.append("BAD\tONLY\tTHREE")

    if rng.random() < 0.08:
        # dense case: tiny word, low-complexity genome and primers -> many hits per seed
        W = rng.choice([3, 4, 5])
        alpha = rng.choice(["AT", "ACG", "GC"])
        sts_lines = []
        for s in range(rng.randint(1, 4)):
            p1 = "".join(rng.choice(alpha) for _ in range(rng.randint(W, 8)))
            p2 = "".join(rng.choice(alpha) for _ in range(rng.randint(W, 8)))
            sts_lines.append(f"D{idx}_{s}\t{p1}\t{p2}\t{rng.randint(10, 60)}\tdense")
        seq = "".join(rng.choice(alpha) for _ in range(rng.randint(100, 700)))
        params = dict(wordsize=W, margin=rng.choice([0, 3, 10]), mismatches=N,
                      three_prime_match=X, iupac_mode=I, default_pcr_size=Z)
        return params, "\n".join(sts_lines) + "\n", [(f">dense{idx}", seq)]

    n_rec = rng.choice([1, 1, 1, 2, 3])
    records = []
    for r in range(n_rec):
        n = rng.choice([0, W - 1, W, W + 1, rng.randint(50, 600), rng.randint(600, 4000)])
        if mode in ("lowcomplex",) or (I and mode in ("iupac", "nruns")):
            n = min(n, 800)
        seq = list(_rand_seq(rng, n, mode))
        # plant amplicons in the orientations merpcr finds
        for p1, p2, size in planted:
            if rng.random() < 0.8 and n > 0:
                prod = max(len(p1) + len(p2), size + rng.randint(-M - 2, M + 2))
                fill = max(0, prod - len(p1) - len(p2))
                form = rng.choice(["plus", "minus", "minus"])
                if form == "plus":
                    a, b = p1, p2
                else:
                    a, b = p2, _rc(p1)
                if N and rng.random() < 0.6:
                    a = _mutate(rng, a, rng.randint(1, N), protect_tail=min(X, len(a)))
                amp = a + _rand_seq(rng, fill, "acgt") + b
                if rng.random() < 0.3:
                    amp = amp.lower()
                start = rng.randint(0, max(0, n - 1))
                if rng.random() < 0.15:
                    start = max(0, n - len(amp) + rng.randint(-5, 5))
                seq[start:start + len(amp)] = list(amp)
        records.append((f">rec{idx}_{r} desc {r}", "".join(seq)))
    params = dict(wordsize=W, margin=M, mismatches=N, three_prime_match=X,
                  iupac_mode=I, default_pcr_size=Z)
    return params, "\n".join(sts_lines) + "\n", records


def gen_fasta_text(rng, records):
    out = []
    if rng.random() < 0.2:
        out.append("ACGTACGT orphan line before header")
    nl = rng.choice(["\n", "\r\n", "\n", "\r"])
    for head, seq in records:
        out.append(head + rng.choice(["", "  ", "\t"]))
        w = rng.choice([60, 70, 13, 1000])
        for i in range(0, len(seq), w):
            chunk = seq[i:i + w]
            if rng.random() < 0.1:
                chunk = chunk + rng.choice([" 123", "*", "  ", "-", "U", "ſ", "\t9"])
            if rng.random() < 0.05:
                out.append("")
            out.append(rng.choice(["", " "]) + chunk)
    return nl.join(out) + nl


# --------------------------------------------------------------------------
# running the reference
# --------------------------------------------------------------------------

def run_ref(params, sts_text, records=None, fasta_text=None, threads=1):
    MerPCR, FASTARecord = _ref()
    eng = MerPCR(threads=threads, **params)
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "x.sts")
        with open(sp, "w") as fh:
            fh.write(sts_text)
        ok = eng.load_sts_file(sp)
        if not ok:
            return {"load_ok": False}
        if fasta_text is not None:
            fp = os.path.join(td, "x.fa")
            with open(fp, "w", newline="") as fh:
                fh.write(fasta_text)
            recs = eng.load_fasta_file(fp)
            loaded = [[r.defline, r.sequence, r.label] for r in recs]
        else:
            recs = [FASTARecord(defline=d, sequence=s) for d, s in records]
            loaded = None
        op = os.path.join(td, "out.txt")
        n = eng.search(recs, op)
        with open(op) as fh:
            out = fh.read()
    res = {"load_ok": True, "n_hits": n, "output": out,
           "max_pcr_size": eng.max_pcr_size,
           "n_records": len(eng.sts_records)}
    if loaded is not None:
        res["fasta"] = loaded
    return res


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__(logging.DEBUG)
        self.msgs = []

    def emit(self, record):
        self.msgs.append([record.levelname, record.getMessage()])


def run_ref_err(params, sts_text, records, threads=1):
    """run_ref for the error paths: the exception type the reference raises from
    load_sts_file or search (if any), the output it wrote before it, and its log lines
    (minus timings)."""
    MerPCR, FASTARecord = _ref()
    cap = _Capture()
    lg = logging.getLogger("merpcr")
    lg.addHandler(cap)
    lg.setLevel(logging.DEBUG)
    res = {}
    try:
        eng = MerPCR(threads=threads, **params)
        with tempfile.TemporaryDirectory() as td:
            sp = os.path.join(td, "x.sts")
            with open(sp, "w") as fh:
                fh.write(sts_text)
            try:
                res["load_ok"] = eng.load_sts_file(sp)
                res["load_error"] = None
            except Exception as e:  # noqa: BLE001 - record the reference's exception type
                res["load_ok"] = None
                res["load_error"] = type(e).__name__
            res["n_records"] = len(eng.sts_records)
            res["keys"] = sorted(eng.sts_table)
            if res["load_ok"]:
                recs = [FASTARecord(defline=d, sequence=s) for d, s in records]
                op = os.path.join(td, "out.txt")
                try:
                    res["n_hits"] = eng.search(recs, op)
                    res["search_error"] = None
                except Exception as e:  # noqa: BLE001
                    res["search_error"] = type(e).__name__
                import gc
                gc.collect()  # the reference leaves its output file to be closed by the collector
                with open(op) as fh:
                    res["output"] = fh.read()
    finally:
        lg.removeHandler(cap)
    res["log"] = [m for m in cap.msgs if " seconds" not in m[1] and not m[1].startswith("Reading STS file")]
    return res


def error_cases(rng):
    """Characters beyond U+00FF (after upper()) in primers and sequences: the reference's
    scode[ord(c)] lookups raise IndexError when the hash or the scan reaches them
    (engine.py:345, 472, 497); characters that upper-case into Latin-1 do not."""
    MerPCR, _ = _ref()
    odd = ["\u03a9", "\u00ff", "\u0131", "\u00df", "\u00e9", "\u017f", "\u4e2d", "\u00b5", "N", "n", "U"]
    kats = []
    for _ in range(400):
        W = rng.randint(3, 12)
        L = rng.randint(0, 24)
        p = "".join(rng.choice(odd) if rng.random() < 0.12 else rng.choice("ACGTacgt") for _ in range(L))
        try:
            r = list(MerPCR(wordsize=W)._hash_value(p))
        except IndexError:
            r = "IndexError"
        kats.append([p, W, r])
    cases = []
    base = "".join(rng.choice("ACGT") for _ in range(3000))
    for i in range(60):
        W = rng.choice([4, 6, 8, 11])
        prm = dict(wordsize=W, margin=rng.choice([0, 5, 50]), mismatches=rng.randint(0, 2), three_prime_match=1,
                   iupac_mode=rng.randint(0, 1), default_pcr_size=240)
        lines = []
        for s in range(rng.randint(1, 4)):
            a = rng.randrange(0, 2500)
            p1 = base[a:a + rng.randint(W, 22)]
            q = a + rng.randint(100, 300)
            p2 = _rc(base[q - rng.randint(W, 22):q])
            if i % 3 == 0 and rng.random() < 0.6:  # an odd character in a primer
                which = rng.choice([0, 1])
                pr = list(p1 if which == 0 else p2)
                pr[rng.randrange(len(pr))] = rng.choice(odd[:8])
                if which == 0:
                    p1 = "".join(pr)
                else:
                    p2 = "".join(pr)
            lines.append(f"S{s}\t{p1}\t{p2}\t{q - a}\tal{s}")
        recs = []
        for r in range(rng.randint(1, 3)):
            s = list(base[rng.randrange(0, 500):][:rng.randint(0, 2500)])
            if i % 3 == 1 and s and rng.random() < 0.5:  # an odd character in a sequence
                s[rng.randrange(len(s))] = rng.choice(odd[:8])
            if i % 3 == 2 and rng.random() < 0.3:  # a short sequence (<= W) with one
                s = [rng.choice(odd[:8])] + list(base[:rng.randint(0, W - 1)])
            recs.append([f">r{r} d", "".join(s)])
        sts = "\n".join(lines) + "\n"
        cases.append({"params": prm, "sts_text": sts, "records": recs, **run_ref_err(prm, sts, recs)})
    return {"hash": kats, "cases": cases}


def unit_kats(rng):
    MerPCR, _ = _ref()
    kat = {"hash": [], "revcomp": [], "compare": [], "pcr_size": []}
    for _ in range(400):
        W = rng.randint(3, 16)
        L = rng.randint(0, 30)
        p = "".join(rng.choice("ACGTUacgtuNRYX-") if rng.random() < 0.15 else rng.choice("ACGT")
                    for _ in range(L))
        kat["hash"].append([p, W, list(MerPCR(wordsize=W)._hash_value(p))])
    eng = MerPCR()
    for _ in range(200):
        s = "".join(rng.choice("ACGTUBDHKMNRSVWXYacgtubdhkmnrsvwxyZ-*1") for _ in range(rng.randint(0, 20)))
        kat["revcomp"].append([s, eng._reverse_complement(s)])
    alpha = "ACGTUacgtuRYMKSWBDHVNXZ-"
    for _ in range(1500):
        L = rng.randint(1, 12)
        a = "".join(rng.choice(alpha) if rng.random() < 0.3 else rng.choice("ACGT") for _ in range(L))
        b = list(a) if rng.random() < 0.7 else [rng.choice("ACGT") for _ in range(L)]
        for _ in range(rng.randint(0, 3)):
            b[rng.randrange(L)] = rng.choice(alpha)
        b = "".join(b)
        if rng.random() < 0.03:
            b = b + "A"
        N = rng.randint(0, 3)
        X = rng.randint(0, 5)
        I = rng.randint(0, 1)
        strand = rng.choice("+-")
        e = MerPCR(mismatches=N, three_prime_match=X, iupac_mode=I)
        kat["compare"].append([a, b, strand, N, X, I, e._compare_seqs(a, b, strand)])
    for f in ["100", "150-250", "0", "-5", "abc", "10-", "-", "1-2-3", "x-y", " 7", "7 ", "3",
              "+9", "1_000", "٣", "100-200", "201-200", "5-5"]:
        kat["pcr_size"].append([f, MerPCR(default_pcr_size=240)._parse_pcr_size(f)])
    return kat


def _plan(n, threads, max_pcr, margin):
    """Chunk plan of the reference's -T N search (same rule as oracle.chunk_plan); used
    only to place amplicons on chunk seams."""
    t = threads if n >= 100000 else 1
    ov = max_pcr + margin - 1
    while t > 1 and (t + 1) * ov > n:
        t -= 1
    size = int((n - (t + 1) * ov) / t) + 2 * ov
    out, off = [], 0
    for i in range(t):
        ln = size if i < t - 1 else n - off
        out.append((off, ln))
        off += ln - ov
    return out


def chunked_cases():
    """-T N corpus: the reference's chunked search (duplicated overlap hits, chunk-local
    record ends) on genomes built so that hits fall on chunk seams."""
    g = random.Random(777)
    out = []

    def acgt(n):
        return "".join(g.choice("ACGT") for _ in range(n))

    def plant(seq, pos, amp):
        return seq[:pos] + amp + seq[pos + len(amp):]

    # 1. planted amplicons on the seams of every T's plan, two orientations
    p1, p2 = "GATTACAGGCTTACCGTA", "CCTAGGATCGATTGCAAT"
    prm = dict(wordsize=11, margin=50, mismatches=1, three_prime_match=1, iupac_mode=0,
               default_pcr_size=240)
    st = f"SEAM\t{p1}\t{p2}\t180\tseam marker\nSEAM2\t{p2}\t{p1}\t200-240\n"
    big = acgt(400000)
    ampf = p1 + acgt(180 - len(p1) - len(p2)) + p2
    ampr = p2 + acgt(190 - len(p1) - len(p2)) + _rc(p1)
    for T in (2, 3, 4, 8):
        for off, ln in _plan(len(big), T, 220, 50)[1:]:    # max_pcr_size = (200+240)//2
            big = plant(big, off + 10, ampf)            # inside the overlap: found twice
            big = plant(big, off + 269 - 60, ampr)      # straddles the previous chunk's end
    small = plant(acgt(60000), 30000, ampf)
    cases = [("seam", prm, st, [(">big seam test", big), (">small", small)], (1, 2, 3, 4, 8))]

    # 2. dense chance hits (W=4, 4-mer primers): many amplicons truncated by chunk ends
    prm2 = dict(wordsize=4, margin=20, mismatches=1, three_prime_match=1, iupac_mode=0,
                default_pcr_size=60)
    st2 = "".join(f"D{i}\t{acgt(g.randint(4, 6))}\t{acgt(g.randint(4, 6))}\t{g.randint(20, 90)}\n"
                  for i in range(4))
    cases.append(("dense", prm2, st2, [(">dense1", acgt(210000)), (">dense2", acgt(100000))], (1, 3, 5)))

    # 3. T reduced by a long product (ov ~ 20k), records at the 100 kbp threshold
    prm3 = dict(wordsize=8, margin=49, mismatches=0, three_prime_match=2, iupac_mode=1,
                default_pcr_size=240)
    q1, q2 = "ACGTTGCAAGGCTA", "TTGACGGCATCAGA"
    st3 = f"LONG\t{q1}\t{q2}\t20000\nSHORT\t{q2}\t{q1}\t150\nIUP\tACGTRYNNACGTAC\tGGCATTYCAGGA\t120\n"
    recs3 = []
    for n in (99999, 100000, 100001, 130000, 250000):
        sq = acgt(n)
        for pos in range(500, n - 300, 21011):
            sq = plant(sq, pos, q2 + acgt(150 - 2 * len(q1)) + q1)         # SHORT '+'
        for pos in range(1700, n - 20100, 17003):
            sq = plant(sq, pos, q1)                                         # LONG '+'
            sq = plant(sq, pos + 20000 - len(q2) + g.randint(-49, 49), q2)
        recs3.append((f">r{n} len={n}", sq))
    cases.append(("reduce", prm3, st3, recs3, (1, 4, 8)))

    for name, prm_, st_, recs, ts in cases:
        outs = {}
        for T in ts:
            r = run_ref(prm_, st_, records=recs, threads=T)
            outs[str(T)] = {"n_hits": r["n_hits"], "output": r["output"]}
            print("chunked", name, T, r["n_hits"], file=sys.stderr)
        out.append({"name": name, "params": prm_, "sts_text": st_, "records": [list(x) for x in recs],
                    "max_pcr_size": r["max_pcr_size"], "by_threads": outs})
    return out


def main():
    if "--errors" in sys.argv:
        erng = random.Random(2026)
        obj = error_cases(erng)
        print("errors: hash raises", sum(k[2] == "IndexError" for k in obj["hash"]),
              "load raises", sum(c["load_error"] is not None for c in obj["cases"]),
              "search raises", sum(bool(c.get("search_error")) for c in obj["cases"]), file=sys.stderr)
        with gzip.open(os.path.join(HERE, "errors.json.gz"), "wt") as fh:
            json.dump(obj, fh, separators=(",", ":"))
        return
    if "--chunked" in sys.argv:
        logging.disable(logging.CRITICAL)
        with gzip.open(os.path.join(HERE, "chunked.json.gz"), "wt") as fh:
            json.dump({"cases": chunked_cases()}, fh, separators=(",", ":"))
        return
    logging.disable(logging.CRITICAL)
    rng = random.Random(20261015)
    sts_path = os.path.join(DATA, "test.sts")
    fa_path = os.path.join(DATA, "test.fa")
    with open(sts_path) as fh:
        sts_text = fh.read()
    with open(fa_path) as fh:
        fa_text = fh.read()

    bundled = []
    variants = [{}, {"mismatches": 1}, {"mismatches": 2}, {"mismatches": 3, "three_prime_match": 0},
                {"iupac_mode": 1, "mismatches": 2}, {"wordsize": 8}, {"wordsize": 16},
                {"wordsize": 8, "mismatches": 3, "margin": 200}, {"margin": 0},
                {"wordsize": 3, "margin": 10}]
    for v in variants:
        params = dict(wordsize=11, margin=50, mismatches=0, three_prime_match=1,
                      iupac_mode=0, default_pcr_size=240)
        params.update(v)
        res = run_ref(params, sts_text, fasta_text=fa_text)
        res.pop("fasta", None)
        bundled.append({"params": params, **res})
        print("bundled", v, res["n_hits"], file=sys.stderr)

    repeat = {"params": dict(wordsize=4, margin=50, mismatches=0, three_prime_match=1,
                             iupac_mode=0, default_pcr_size=240),
              "sts_text": "REPEAT\tATCG\tCGAT\t20\n",
              "records": [[">repeat", "ATCGCGAT" * 1000]]}
    r = run_ref(repeat["params"], repeat["sts_text"], records=repeat["records"])
    repeat.update(r)
    repeat["sha256"] = hashlib.sha256(r["output"].encode()).hexdigest()
    print("repeat", r["n_hits"], repeat["sha256"][:16], file=sys.stderr)

    cases = []
    for i in range(700):
        params, sts, recs = gen_case(rng, i)
        use_fasta = rng.random() < 0.25
        if use_fasta:
            ft = gen_fasta_text(rng, recs)
            res = run_ref(params, sts, fasta_text=ft)
            case = {"params": params, "sts_text": sts, "fasta_text": ft, **res}
        else:
            res = run_ref(params, sts, records=recs)
            case = {"params": params, "sts_text": sts, "records": [list(x) for x in recs], **res}
        cases.append(case)
    tot = sum(c.get("n_hits", 0) for c in cases)
    print("random cases", len(cases), "hits", tot, file=sys.stderr)

    # IUPAC N-run explosion and record-end truncation, hand-built
    special = []
    p1, p2 = "ACGTTGCAAGCTTAGC", "GGATCCTTAGGCATCA"
    seq = "ACGT" * 10 + p1 + "N" * 300 + "ACGT" * 10
    for I in (0, 1):
        prm = dict(wordsize=11, margin=50, mismatches=0, three_prime_match=1, iupac_mode=I,
                   default_pcr_size=240)
        st = f"NRUN\t{p1}\t{p2}\t200\n"
        special.append({"params": prm, "sts_text": st, "records": [[">nrun", seq]],
                        **run_ref(prm, st, records=[(">nrun", seq)])})
    g = random.Random(7)
    body = "".join(g.choice("ACGT") for _ in range(300))
    tail = p2 + "".join(g.choice("ACGT") for _ in range(60)) + _rc(p1)
    for cut in range(0, 40, 3):
        s = body + tail[:len(tail) - cut] if cut else body + tail
        prm = dict(wordsize=8, margin=50, mismatches=1, three_prime_match=1, iupac_mode=0,
                   default_pcr_size=240)
        st = f"END\t{p1}\t{p2}\t150\n"
        special.append({"params": prm, "sts_text": st, "records": [[">end", s]],
                        **run_ref(prm, st, records=[(">end", s)])})

    # T>1 chunking artefacts (documentation of reference behaviour, not a parity target)
    threaded = []
    g = random.Random(11)
    big = "".join(g.choice("ACGT") for _ in range(400000))
    pp1, pp2 = "TTGACCGATAGCTAGGCA", "CATGCTAGGATCCAGTTA"
    amp = pp2 + "".join(g.choice("ACGT") for _ in range(164)) + _rc(pp1)
    big = list(big)
    for pos in (1000, 99950, 199880, 299830, 399700):
        big[pos:pos + len(amp)] = list(amp)
    big = "".join(big)
    prm = dict(wordsize=11, margin=50, mismatches=0, three_prime_match=1, iupac_mode=0,
               default_pcr_size=240)
    st = f"CHUNK\t{pp1}\t{pp2}\t200\n"
    for T in (1, 4):
        threaded.append({"params": prm, "threads": T, "sts_text": st,
                         "records": [[">big", big]],
                         **run_ref(prm, st, records=[(">big", big)], threads=T)})
        print("threaded", T, threaded[-1]["n_hits"], file=sys.stderr)

    kats = unit_kats(rng)

    def dump(name, obj):
        with gzip.open(os.path.join(HERE, name), "wt") as fh:
            json.dump(obj, fh, separators=(",", ":"))

    dump("bundled.json.gz", {"sts_sha256": hashlib.sha256(sts_text.encode()).hexdigest(),
                             "fa_sha256": hashlib.sha256(fa_text.encode()).hexdigest(),
                             "cases": bundled})
    dump("repeat.json.gz", repeat)
    dump("random_cases.json.gz", {"cases": cases})
    dump("special_cases.json.gz", {"cases": special})
    dump("threaded.json.gz", {"cases": threaded})
    dump("unit_kats.json.gz", kats)


if __name__ == "__main__":
    main()
