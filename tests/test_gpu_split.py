"""Split seeds (W 7..9, I = 0, N <= 1; mp_internal.h kSplitSpan) against the C oracle.

The dense table's search runs as a scan of the exact seed [0, 11), a scan of the gapped
seed [0, W) ++ [11, S) (N = 1; S = 22 - W, a = 11 - W) and a dense scan of the records
neither can carry.  The cases plant amplicons whose one mismatch sits in A = [W, 11), in
B = [11, S) or past S (inside the gapped seed's post bases), invalid genome bases (N, IUPAC)
and U inside A, records that stay with the dense scan (seed inside the primer, IUPAC bases,
short primers) and keys shared by many records.
Every hit list must equal the C oracle's byte for byte, with the split on and off.
"""
import tempfile

import numpy as np
import pytest

from merpcr_amd import FASTARecord, MerPCR
from oracle import epcr_oracle as O

pytestmark = pytest.mark.gpu


def _case(W, N, seed):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)

    def rnd(n):
        return acgt[rng.integers(0, 4, n)].tobytes().decode()

    lines = []
    prefixes = [rnd(16) for _ in range(5)]
    for i in range(1200):
        l1, l2 = int(rng.integers(17, 26)), int(rng.integers(17, 26))
        p1, p2 = rnd(l1), rnd(l2)
        kind = i % 12
        S = 22 - W
        if kind in (0, 1):            # shared 16-base prefixes: multi-record buckets in both seeds
            p1 = prefixes[i % 5] + p1[16:]
        elif kind == 2:               # shared W-mer only: one dense key, distinct seeds
            p1 = prefixes[i % 5][:W] + p1[W:]
        elif kind == 3:               # IUPAC base inside [W, S + 3): the rest table
            j = W + int(rng.integers(0, S + 3 - W))
            p1 = p1[:j] + "RYKMSWN"[i % 7] + p1[j + 1:]
        elif kind == 4:               # seed inside the primer: the rest table
            p1 = "N" + p1[1:]
        elif kind == 5:               # shorter than S + post (N = 1) / 11 (N = 0)
            p1 = p1[:W + int(rng.integers(0, S + 3 - W))]
        lines.append(f"S{i}\t{p1}\t{p2}\t{int(rng.integers(80, 300))}\n")
    sts_text = "".join(lines)
    glen = 900_000
    g = acgt[rng.integers(0, 4, glen)].copy()
    for i in range(0, 1200, 2):
        _, p1, p2, size = lines[i].rstrip("\n").split("\t")[:4]
        a = "".join(c if c in "ACGT" else "G" for c in p1)
        b = O.revcomp(a)
        for x, y in ((a, p2), (p2, b)):
            x = list(x)
            where = int(rng.integers(0, 7))  # independent of the record kind: single- and multi-record buckets
            a_len = 11 - W
            if len(x) >= S + 3:
                if where == 0:    # one mismatch in A = [W, 11)
                    j = W + int(rng.integers(0, a_len))
                    x[j] = "ACGT"[("ACGT".index(x[j]) + 1) % 4]
                elif where == 1:  # one mismatch in B = [11, S)
                    j = 11 + int(rng.integers(0, a_len))
                    x[j] = "ACGT"[("ACGT".index(x[j]) + 2) % 4]
                elif where == 2:  # an invalid genome base in A
                    x[W + int(rng.integers(0, a_len))] = "NRY"[i % 3]
                elif where == 3:  # U in A (a T there reads as T in the seeds)
                    x[W + int(rng.integers(0, a_len))] = "U"
                elif where == 4:  # mismatches in both halves
                    x[W] = "ACGT"[("ACGT".index(x[W]) + 1) % 4]
                    x[S - 1] = "ACGT"[("ACGT".index(x[S - 1]) + 1) % 4]
                elif where == 5:  # one mismatch in A and one in the post bases after S
                    x[W] = "ACGT"[("ACGT".index(x[W]) + 3) % 4]
                    j = S + int(rng.integers(0, 2))
                    x[j] = "ACGT"[("ACGT".index(x[j]) + 1) % 4]
            x = "".join(x)
            amp = (x + rnd(max(int(size) - len(x) - len(y), 0)) + y).encode()
            st = int(rng.integers(0, glen - len(amp)))
            g[st:st + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    for c, frac in ((b"N", 0.003), (b"R", 0.001), (b"U", 0.002), (b"a", 0.05)):
        idx = rng.integers(0, glen, int(glen * frac))
        g[idx] = c[0]
    return sts_text, g


@pytest.mark.parametrize("W,N", [(7, 1), (8, 1), (9, 1), (8, 0), (9, 0)])
def test_split_seeds_vs_c_oracle(W, N):
    from oracle import c_oracle as C
    sts_text, g = _case(W, N, 40 + W * 2 + N)
    prm = dict(wordsize=W, mismatches=N, iupac_mode=0, margin=50, three_prime_match=1)
    table = O.load_sts_lines(sts_text.splitlines(True), W, 240)
    ref = C.search(table, [g], O.params(**prm), 8)
    assert len(ref) > (150 if N else 10)
    seq = g.tobytes().decode("ascii")
    stats = {}
    for split in (True, False):
        eng = MerPCR(**prm)
        eng.search_options = dict(split=split)
        with tempfile.TemporaryDirectory() as td:
            p = f"{td}/x.sts"
            with open(p, "w") as fh:
                fh.write(sts_text)
            assert eng.load_sts_file(p)
        hits = eng.find_hits([FASTARecord(defline=">chrS", sequence=seq)])
        assert len(hits) == len(ref) and hits.tobytes() == ref.tobytes(), split
        stats[split] = dict(eng.last_search_stats)
        sp = eng.device_table().split()
        assert sp["seed_tables"] == (2 if N else 1), sp
        assert 0 < sp["rest_records"] < len(eng.sts_records) // 2, sp  # kinds 3-5 stay dense
    # the split scans count other candidates than the dense scan: the two paths really differ
    assert stats[True]["candidates"] != stats[False]["candidates"], stats


def test_split_sharded_ranges():
    """Owned (seq, k) ranges through the split scans concatenate to the whole list."""
    from merpcr_amd import _native
    sts_text, g = _case(8, 1, 7)
    eng = MerPCR(wordsize=8, mismatches=1)
    with tempfile.TemporaryDirectory() as td:
        p = f"{td}/x.sts"
        with open(p, "w") as fh:
            fh.write(sts_text)
        assert eng.load_sts_file(p)
    seq = g.tobytes().decode("ascii")
    seqs = [seq[:400_000], seq[400_000:400_700], seq[400_700:]]
    data = eng.encode_sequences(seqs)
    genome = _native.Genome(0, [len(d) for d in data])
    for i, d in enumerate(data):
        genome.put(i, d)
    genome.seal()
    s = _native.Search(eng.device_table(), genome)
    whole = s.fetch(s.run())
    cuts = [(0, 0), (0, 123_457), (1, 300), (2, 0), (2, 250_001), (3, 0)]
    parts = [s.fetch(s.run((a, b, ka, kb))) for (a, ka), (b, kb) in zip(cuts[:-1], cuts[1:])]
    assert len(whole) > 100
    assert np.array_equal(np.concatenate(parts), whole)


@pytest.mark.parametrize("W,N,I", [(6, 1, 0), (8, 2, 0), (8, 1, 1), (10, 1, 0)])
def test_no_split_outside_its_domain(W, N, I):
    """W 7..9, I = 0, N <= 1 only: other tables keep their own scan (and say so)."""
    sts_text, _ = _case(8, 1, 3)
    eng = MerPCR(wordsize=W, mismatches=N, iupac_mode=I, margin=50)
    with tempfile.TemporaryDirectory() as td:
        p = f"{td}/x.sts"
        with open(p, "w") as fh:
            fh.write(sts_text)
        assert eng.load_sts_file(p)
    assert eng.device_table().split()["seed_tables"] == 0
