"""CPU oracle for the merpcr STS-search hot path.  TEST INFRASTRUCTURE ONLY.

This module is a plain-Python restatement of the algorithm that
FOI-Bioinformatics/merpcr runs on its search path.  It exists only to check the
HIP implementation: nothing under ``merpcr_amd/`` may import it, and the product
path never routes through it.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg use it.

Parity pinning: this restatement is checked against golden vectors produced by
running the reference itself in the survey/build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.json.gz``) and against the
known-answer values held by the reference's own tests (see
``tests/test_oracle_golden.py``).

Every function cites the reference file:line it restates (paths relative to the
reference repository root, ``src/merpcr/...``).
"""

from __future__ import annotations

import bisect
from typing import Dict, List, Optional, Sequence, Tuple

# --------------------------------------------------------------------------
# Alphabet tables
# --------------------------------------------------------------------------

# core/engine.py:99-109 -- A/C/G/T and U (RNA, treated as T) carry a 2-bit
# code, every other character is "ambiguous" for hashing purposes.
_BASE2 = {"A": 0, "C": 1, "G": 2, "T": 3, "U": 3}

# core/engine.py:112-135 -- complement map used by the reverse complement.
# Case is preserved; any character not in the map becomes 'N'.
_COMPL_UP = {
    "A": "T", "C": "G", "G": "C", "T": "A", "U": "A",
    "B": "V", "V": "B", "D": "H", "H": "D", "K": "M", "M": "K",
    "R": "Y", "Y": "R", "N": "N", "S": "S", "W": "W", "X": "X",
}
_COMPL = dict(_COMPL_UP)
_COMPL.update({k.lower(): v.lower() for k, v in _COMPL_UP.items()})

# core/engine.py:138-172 -- IUPAC expansion sets.  Two characters that both
# appear here match iff their expansions intersect; that is exactly the
# intersection of the 4-bit base masks below (A=1, C=2, G=4, T=U=8).
IUPAC_MASK = {
    "A": 1, "C": 2, "G": 4, "T": 8, "U": 8,
    "R": 5, "Y": 10, "M": 3, "K": 12, "S": 6, "W": 9,
    "B": 14, "D": 13, "H": 11, "V": 7, "N": 15,
}

# io/fasta.py:60 -- characters that survive the FASTA line filter
# (``c.upper() in "ACGTBDHKMNRSVWXY"``).  Enumerated over all of Unicode:
# the 32 ASCII letters plus U+017F (LATIN SMALL LETTER LONG S, upper = 'S').
FASTA_KEEP = frozenset("ABCDGHKMNRSTVWXYabcdghkmnrstvwxyſ")

# Engine defaults and bounds, core/engine.py:17-39.
DEFAULTS = dict(wordsize=11, margin=50, mismatches=0, three_prime_match=1,
                iupac_mode=0, default_pcr_size=240, threads=1)
MIN_FILESIZE_FOR_THREADING = 100000


# --------------------------------------------------------------------------
# Primer helpers
# --------------------------------------------------------------------------

def hash_word(primer: str, W: int) -> Tuple[int, int]:
    """First all-ACGTU W-mer of ``primer`` -> (offset, 2W-bit value).

    Restates ``MerPCR._hash_value`` (core/engine.py:331-355): the primer is
    upper-cased, the first offset whose W characters all have a 2-bit code is
    chosen, and the value packs the first base into the most significant bits.
    (-1, 0) when the primer is shorter than W or has no such window.  Like the
    reference's ``self.scode[ord(base)]`` (a 256-entry list, engine.py:345), a
    character beyond U+00FF raises IndexError when the loop reaches it.
    """
    p = primer.upper()
    if len(p) < W:
        return -1, 0
    for off in range(len(p) - W + 1):
        v = 0
        for ch in p[off:off + W]:
            if ord(ch) > 0xFF:
                raise IndexError("list index out of range")
            c = _BASE2.get(ch)
            if c is None:
                break
            v = (v << 2) | c
        else:
            return off, v
    return -1, 0


def revcomp(s: str) -> str:
    """Reverse complement, core/engine.py:357-359 (table 112-135)."""
    return "".join(_COMPL.get(ch, "N") for ch in reversed(s))


def parse_pcr_size(field: str, default: int) -> int:
    """PCR size field -> int, restating core/engine.py:304-322.

    'a-b' -> (a+b)//2 when split gives exactly two non-empty ints, otherwise the
    default; a plain int > 0 is taken as is; anything else -> default.
    """
    if "-" in field:
        parts = field.split("-")
        if len(parts) == 2 and parts[0] and parts[1]:
            try:
                return (int(parts[0]) + int(parts[1])) // 2
            except ValueError:
                return default
        return default
    try:
        v = int(field)
    except ValueError:
        return default
    return v if v > 0 else default


class OracleRecord:
    """One oriented STS record (the '+' or '-' entry of core/engine.py:253-281)."""

    __slots__ = ("sts_id", "primer1", "primer2", "pcr_size", "alias",
                 "line_no", "hash_offset", "direct", "key")

    def __init__(self, sts_id, primer1, primer2, pcr_size, alias, line_no,
                 hash_offset, direct, key):
        self.sts_id = sts_id
        self.primer1 = primer1
        self.primer2 = primer2
        self.pcr_size = pcr_size
        self.alias = alias
        self.line_no = line_no
        self.hash_offset = hash_offset
        self.direct = direct
        self.key = key


class OracleTable:
    """STS records in insertion order plus the key -> [record index] map."""

    def __init__(self):
        self.records: List[OracleRecord] = []
        self.buckets: Dict[int, List[int]] = {}
        self.max_pcr_size = 0

    def add(self, rec: OracleRecord):
        # core/engine.py:324-329: append to the bucket and to the flat list.
        self.buckets.setdefault(rec.key, []).append(len(self.records))
        self.records.append(rec)


def load_sts_lines(lines: Sequence[str], W: int,
                   default_pcr_size: int) -> Optional[OracleTable]:
    """Build the seed table from STS lines, restating core/engine.py:193-302.

    Returns None where the reference's ``load_sts_file`` returns False because
    a non-comment line has fewer than four tab-separated fields.
    """
    t = OracleTable()
    for idx, raw in enumerate(lines):
        line_no = idx + 1
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        f = line.split("\t")
        if len(f) < 4:
            return None
        p1 = f[1].upper()
        p2 = f[2].upper()
        size = parse_pcr_size(f[3], default_pcr_size)
        alias = f[4] if len(f) > 4 else ""
        if len(p1) < W or len(p2) < W:
            continue
        if len(p1) + len(p2) > size:
            size = len(p1) + len(p2)
        if size > t.max_pcr_size:
            t.max_pcr_size = size
        off1, key1 = hash_word(p1, W)
        if off1 >= 0:
            t.add(OracleRecord(f[0], p1, p2, size, alias, line_no, off1, "+", key1))
        rc1 = revcomp(p1)
        off2, key2 = hash_word(p2, W)
        if off2 >= 0:
            t.add(OracleRecord(f[0], p2, rc1, size, alias, line_no, off2, "-", key2))
    return t


def read_lines_like_python(path: str) -> List[str]:
    """``open(path).readlines()`` as the reference does (text mode)."""
    with open(path, "r") as fh:
        return fh.readlines()


# --------------------------------------------------------------------------
# FASTA
# --------------------------------------------------------------------------

def fasta_from_lines(lines) -> List[Tuple[str, str]]:
    """(defline, filtered sequence) pairs, restating io/fasta.py:38-66."""
    out = []
    head = None
    parts: List[str] = []
    for raw in lines:
        line = raw.strip()
        if not line:
            continue
        if line.startswith(">"):
            if head is not None:
                out.append((head, "".join(parts)))
            head = line
            parts = []
        else:
            parts.append("".join(ch for ch in line if ch in FASTA_KEEP))
    if head is not None:
        out.append((head, "".join(parts)))
    return out


def fasta_label(defline: str) -> str:
    """First whitespace token of the defline, core/models.py:40-49."""
    d = defline.strip()[1:] if ">" in defline else defline.strip()
    return d.split()[0]


# --------------------------------------------------------------------------
# Primer comparison
# --------------------------------------------------------------------------

def primer_match(seg: str, primer: str, strand: str, N: int, X: int, I: int) -> bool:
    """Mismatch-tolerant compare, restating core/engine.py:599-642.

    A position is 3'-protected when strand is '+' and i >= L-X, or strand is
    '-' and i < X.  Any protected mismatch, or more than N mismatches, fails.
    """
    L = len(seg)
    if L != len(primer):
        return False
    mm = 0
    for i in range(L):
        a = seg[i].upper()
        b = primer[i].upper()
        if I:
            ma = IUPAC_MASK.get(a)
            mb = IUPAC_MASK.get(b)
            ok = (ma & mb) != 0 if (ma is not None and mb is not None) else a == b
        else:
            ok = a == b
        if not ok:
            if (strand == "+" and i >= L - X) or (strand == "-" and i < X):
                return False
            mm += 1
            if mm > N:
                return False
    return True


# --------------------------------------------------------------------------
# Scan of one sequence (one chunk in the reference's terms)
# --------------------------------------------------------------------------

def try_order(lo: int, hi: int, M: int):
    """Amplicon-end offsets in the reference's try order, core/engine.py:542-593.

    d = 0 first, then for i = 1..M: -i if i <= lo, then +i if i <= hi.
    """
    yield 0
    for i in range(1, M + 1):
        if i <= lo:
            yield -i
        if i <= hi:
            yield i


def try_rank(d: int) -> int:
    """Rank of offset d in ``try_order``: 0, 1 for -1, 2 for +1, 3 for -2 ..."""
    if d == 0:
        return 0
    return 2 * (-d) - 1 if d < 0 else 2 * d


def match_at(s: str, n: int, k: int, rec: OracleRecord, p: dict, out: list, rec_idx: int):
    """Primer-1 verify and amplicon pair-check, restating core/engine.py:507-597.

    Appends (pos1, pos2, rec_idx) for every offset whose primer-2 compare passes.
    """
    l1 = len(rec.primer1)
    if k + l1 > n or not primer_match(s[k:k + l1], rec.primer1, "+",
                                      p["mismatches"], p["three_prime_match"],
                                      p["iupac_mode"]):
        return
    l2 = len(rec.primer2)
    avail = n - (k + l1)
    if avail < l2:
        return
    e = rec.pcr_size
    if e > avail + l1:
        e = avail + l1
        hi = 0
    else:
        hi = min(p["margin"], n - k - e)
    lo = max(0, min(p["margin"], e - l1 - l2))
    for d in try_order(lo, hi, p["margin"]):
        p2 = k + e - l2 + d
        if d <= 0 and k + l1 > p2:
            continue
        if p2 + l2 > n:
            continue
        if primer_match(s[p2:p2 + l2], rec.primer2, "-", p["mismatches"],
                        p["three_prime_match"], p["iupac_mode"]):
            out.append((k, p2 + l2 - 1, rec_idx))


def scan_sequence(seq: str, table: OracleTable, p: dict) -> List[Tuple[int, int, int]]:
    """All hits of one sequence in discovery order, restating core/engine.py:453-505.

    Hits are (pos1, pos2, record index), 0-based and relative to ``seq``.  A
    window is seeded iff its W characters are all A/C/G/T/U (the countdown at
    engine.py:464-503 is exactly that test).
    """
    s = seq.upper()
    n = len(s)
    W = p["wordsize"]
    out: List[Tuple[int, int, int]] = []
    if n <= W:
        return out
    if not s.isascii() and max(map(ord, s)) > 0xFF:
        # engine.py:472/497 look every base up in the 256-entry scode list
        raise IndexError("list index out of range")
    mask = (1 << (2 * W)) - 1
    h = 0
    last_bad = -1  # index of the last non-ACGTU character seen
    for j in range(n):
        c = _BASE2.get(s[j])
        if c is None:
            last_bad = j
            h = (h << 2) & mask
        else:
            h = ((h << 2) | c) & mask
        pos = j - W + 1
        if pos < 0 or last_bad >= pos:
            continue
        bucket = table.buckets.get(h)
        if bucket is None:
            continue
        for ri in bucket:
            rec = table.records[ri]
            k = pos - rec.hash_offset
            if k >= 0 and k + len(rec.primer1) <= n:
                match_at(s, n, k, rec, p, out, ri)
    return out


def canonical_sort_key(hit, table: OracleTable, n: int, p: dict):
    """Total order equal to the reference's T'=1 output order.

    (pos1, hash_offset, record index, try rank); the stable sort by pos1 at
    core/engine.py:434 over discovery order yields exactly this order.
    """
    k, pos2, ri = hit
    rec = table.records[ri]
    l2 = len(rec.primer2)
    e = rec.pcr_size if rec.pcr_size <= n - k else n - k
    d = (pos2 + 1 - l2) - (k + e - l2)
    return (k, rec.hash_offset, ri, try_rank(d))


# --------------------------------------------------------------------------
# Whole search (one output line per hit)
# --------------------------------------------------------------------------

def chunk_plan(n: int, threads: int, max_pcr_size: int, margin: int):
    """(offset, length) chunks, restating core/engine.py:380-411."""
    t = threads if n >= MIN_FILESIZE_FOR_THREADING else 1
    ov = max_pcr_size + margin - 1
    while t > 1 and (t + 1) * ov > n:
        t -= 1
    size = int((n - (t + 1) * ov) / t) + 2 * ov
    plan = []
    off = 0
    for i in range(t):
        ln = size if i < t - 1 else n - off
        plan.append((off, ln))
        off += ln - ov
    return plan


def search_lines(records: Sequence[Tuple[str, str]], table: OracleTable, p: dict,
                 threads: int = 1) -> List[str]:
    """Output lines of ``MerPCR.search``, restating core/engine.py:365-451.

    ``records`` are (label, sequence).  threads > 1 reproduces the reference's
    chunked semantics (each chunk scanned as its own sequence, chunk results
    concatenated in chunk order, then a stable sort on pos1).
    """
    lines = []
    for label, seq in records:
        n = len(seq)
        hits = []
        for off, ln in chunk_plan(n, threads, table.max_pcr_size, p["margin"]):
            for k, pos2, ri in scan_sequence(seq[off:off + ln], table, p):
                hits.append((k + off, pos2 + off, ri))
        hits.sort(key=lambda h: h[0])
        for k, pos2, ri in hits:
            r = table.records[ri]
            lines.append(f"{label}\t{k + 1}..{pos2 + 1}\t{r.sts_id}\t{r.alias}\t({r.direct})")
    return lines


def scan_chunk(task) -> List[Tuple[int, int, int]]:
    """One ProcessPool work item of the reference's -T N execution model
    (engine.py:412-422: each chunk is scanned as a sequence of its own by a worker
    process that receives the pickled table); hits shifted to record coordinates."""
    seq, off, table, p = task
    return [(k + off, pos2 + off, ri) for k, pos2, ri in scan_sequence(seq, table, p)]


def params(**kw) -> dict:
    p = dict(DEFAULTS)
    p.update(kw)
    return p
