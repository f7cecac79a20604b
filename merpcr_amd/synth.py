"""Synthetic STS sets and chromosome-scale genomes for the benchmark configs.

BASELINE.json configs:
  c2  10k STS  vs one 250 Mbp chromosome, W=11 N=0
  c3  100k STS vs 3 Gbp human-size genome (24 records), W=11 N=1 M=50   <- bench default
  c4  100k degenerate STS (~10% IUPAC positions) vs 3 Gbp, I=1 N=2
  c5  100k STS vs 3 Gbp, W=8 N=1 (seed-table saturation)
Genome: iid uniform ACGT, 30% soft-masked (lower case) in 1 kbp blocks, ~5% N in
runs of 100 bp - 50 kbp.  Every STS is planted once in each orientation merpcr
finds ('+': p1 .. p2 literal; '-': p2 .. revcomp(p1)), with product length
size +- U(0, M) and, for N > 0, mismatches placed outside the seed window and
the 3'-protected bases, so the true hit count is known (about 2 per STS).
The genome is generated directly in device memory with torch (plumbing only).
"""

from __future__ import annotations

import dataclasses
from typing import List, Optional

import numpy as np

# GRCh38 primary chromosome lengths (Mbp), scaled to the requested total
_HUMAN_MBP = [248.9, 242.2, 198.3, 190.2, 181.5, 170.8, 159.3, 145.1, 138.4, 133.8, 135.1, 133.3,
              114.4, 107.0, 102.0, 90.3, 83.3, 80.4, 58.6, 64.4, 46.7, 50.8, 156.0, 57.2]
_NAMES = [f"chr{i}" for i in range(1, 23)] + ["chrX", "chrY"]
_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTRYMKSWBDHVN", b"TGCAYRKMSWVHDBN"):
    _COMP[_a] = _b

CONFIGS = {
    "c1": dict(n_sts=0, total=0, W=11, N=0, M=50, I=0, records=0, nrun=0.0, iupac=0.0),
    "c2": dict(n_sts=10_000, total=250_000_000, W=11, N=0, M=50, I=0, records=1, nrun=0.0, iupac=0.0),
    "c3": dict(n_sts=100_000, total=3_000_000_000, W=11, N=1, M=50, I=0, records=24, nrun=0.05, iupac=0.0),
    "c4": dict(n_sts=100_000, total=3_000_000_000, W=11, N=2, M=50, I=1, records=24, nrun=0.05, iupac=0.10),
    "c5": dict(n_sts=100_000, total=3_000_000_000, W=8, N=1, M=50, I=0, records=24, nrun=0.05, iupac=0.0),
}


@dataclasses.dataclass
class STSSet:
    ids: List[str]
    p1: List[bytes]
    p2: List[bytes]
    size: np.ndarray
    fields: List[str]

    def text(self) -> str:
        return "".join(f"{i}\t{a.decode()}\t{b.decode()}\t{f}\tsynthetic\n"
                       for i, a, b, f in zip(self.ids, self.p1, self.p2, self.fields))


def revcomp(b: bytes) -> bytes:
    return _COMP[np.frombuffer(b, dtype=np.uint8)[::-1]].tobytes()


def make_sts(n: int, seed: int = 2, W: int = 11, iupac: float = 0.0) -> STSSet:
    """n primer pairs: lengths U[18,25], sizes U[100,400] (10% as 'a-b' ranges)."""
    rng = np.random.default_rng(seed)
    L1 = rng.integers(18, 26, n)
    L2 = rng.integers(18, 26, n)
    size = rng.integers(100, 401, n)
    codes = np.frombuffer(b"RYSWKMN", dtype=np.uint8)
    ids, p1s, p2s, fields = [], [], [], []
    for i in range(n):
        a = _ACGT[rng.integers(0, 4, L1[i])]
        b = _ACGT[rng.integers(0, 4, L2[i])]
        if iupac > 0:
            # keep the first W bases (the seed window) and the 3'-most 3 bases plain
            for p in (a, b):
                span = np.arange(W, len(p) - 3)
                if len(span):
                    m = span[rng.random(len(span)) < iupac * len(p) / len(span)]
                    p[m] = codes[rng.integers(0, len(codes), len(m))]
        ids.append(f"SYN{i:06d}")
        p1s.append(a.tobytes())
        p2s.append(b.tobytes())
        if rng.random() < 0.1:
            r = int(rng.integers(1, 30))
            fields.append(f"{size[i] - r}-{size[i] + r}")
        else:
            fields.append(str(int(size[i])))
    return STSSet(ids, p1s, p2s, size, fields)


def layout(total: int, records: int):
    """Record names and lengths: human-like proportions summing to `total`."""
    if records <= 1:
        return ["chr1"], [int(total)]
    w = np.array((_HUMAN_MBP * ((records + 23) // 24))[:records])
    lens = np.floor(w / w.sum() * total).astype(np.int64)
    lens[0] += total - lens.sum()
    names = (_NAMES * ((records + 23) // 24))[:records]
    return names, [int(x) for x in lens]


def _mutate(rng, p: bytes, k: int, lo: int, hi: int) -> bytes:
    a = bytearray(p)
    for _ in range(k):
        if hi <= lo:
            break
        i = int(rng.integers(lo, hi))
        a[i] = int(_ACGT[(np.searchsorted(_ACGT, a[i]) + int(rng.integers(1, 4))) % 4]) if a[i] in b"ACGT" else a[i]
    return bytes(a)


_SETS = {ord(k): np.frombuffer(v, dtype=np.uint8) for k, v in
         {"R": b"AG", "Y": b"CT", "M": b"AC", "K": b"GT", "S": b"CG", "W": b"AT", "B": b"CGT",
          "D": b"AGT", "H": b"ACT", "V": b"ACG", "N": b"ACGT"}.items()}


def _concrete(rng, p: bytes) -> bytes:
    """Genome bytes for a degenerate primer: each IUPAC code -> one base it allows."""
    a = bytearray(p)
    for i, c in enumerate(a):
        s = _SETS.get(c)
        if s is not None:
            a[i] = int(s[int(rng.integers(0, len(s)))])
    return bytes(a)


def amplicons(sts: STSSet, total: int, seed: int, N: int, M: int, W: int):
    """Planted amplicon bytes and their global start positions (disjoint slots)."""
    rng = np.random.default_rng(seed + 100)
    n = len(sts.ids)
    amps = []
    for i in range(n):
        p1, p2, size = sts.p1[i], sts.p2[i], int(sts.size[i])
        for form in (0, 1):
            a, b = (p1, p2) if form == 0 else (p2, revcomp(p1))
            a, b = _concrete(rng, a), _concrete(rng, b)
            if N:
                a = _mutate(rng, a, int(rng.integers(1, N + 1)), W, len(a) - 1)
            prod = max(len(a) + len(b), size + int(rng.integers(-M, M + 1)))
            fill = _ACGT[rng.integers(0, 4, prod - len(a) - len(b))].tobytes()
            amps.append(a + fill + b)
    slots = len(amps)
    slot = total // max(slots, 1)
    starts = np.arange(slots, dtype=np.int64) * slot
    lens = np.array([len(x) for x in amps], dtype=np.int64)
    room = np.maximum(slot - lens, 1)
    starts += (rng.random(slots) * room).astype(np.int64)
    order = rng.permutation(slots)  # spread STS across the genome
    return [amps[j] for j in order], starts


def build_genome_torch(total: int, records: int, sts: Optional[STSSet], seed: int, N: int, M: int, W: int,
                       nrun: float, device, lens: Optional[List[int]] = None):
    """(names, lengths, uint8 device buffer with records at 64-aligned offsets, offsets).

    `lens` overrides the human-like layout (record lengths summing to `total`)."""
    import torch
    if lens is None:
        names, lens = layout(total, records)
    else:
        lens = [int(x) for x in lens]
        assert sum(lens) == total and len(lens) == records, (lens, total, records)
        names = [f"rec{i}" for i in range(records)]
    offs = np.zeros(len(lens), dtype=np.int64)
    pos = 0
    for i, n in enumerate(lens):
        offs[i] = pos
        pos += (n + 63) // 64 * 64
    buf = torch.empty(pos + 64, dtype=torch.uint8, device=device)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    chunk = 1 << 28
    rng = np.random.default_rng(seed + 7)
    for r, n in enumerate(lens):
        o = int(offs[r])
        for c in range(0, n, chunk):
            m = min(chunk, n - c)
            idx = torch.randint(0, 4, (m,), dtype=torch.uint8, device=device, generator=gen)
            buf[o + c:o + c + m] = lut[idx.long()]
            del idx
    # concatenated view of all records in genome coordinates -> buffer offsets
    rec_start = np.cumsum([0] + lens[:-1])

    def to_buf(g):  # genome coordinate -> buffer index
        r = np.searchsorted(rec_start, g, side="right") - 1
        return offs[r] + (g - rec_start[r]), r

    # N runs (human-like: 100 bp .. 50 kbp), ~nrun of the genome
    if nrun > 0:
        target = int(total * nrun)
        covered = 0
        while covered < target:
            ln = int(min(50_000, max(100, rng.lognormal(8.5, 1.5))))
            g = int(rng.integers(0, total - ln))
            b, r = to_buf(g)
            end = min(int(b) + ln, int(offs[r]) + lens[r])
            buf[int(b):end] = ord("N")
            covered += end - int(b)
    planted = None
    if sts is not None and len(sts.ids):
        amps, starts = amplicons(sts, total, seed, N, M, W)
        ends = starts + np.array([len(a) for a in amps])
        b0, r0 = to_buf(starts)
        # drop amplicons that would straddle a record boundary, and any that overlaps an
        # earlier-starting kept one (a scatter with duplicate indices has no defined
        # winner on the GPU, which made the genome differ between processes)
        keep = (starts - rec_start[r0] + (ends - starts)) <= np.array(lens)[r0]
        last_end = -1
        for i in np.argsort(starts, kind="stable"):
            if not keep[i]:
                continue
            if starts[i] < last_end:
                keep[i] = False
            else:
                last_end = ends[i]
        amps = [a for a, k in zip(amps, keep) if k]
        b0 = b0[keep]
        data = np.frombuffer(b"".join(amps), dtype=np.uint8)
        alens = np.array([len(a) for a in amps], dtype=np.int64)
        first = np.repeat(b0 - np.concatenate([[0], np.cumsum(alens)[:-1]]), alens)
        idx = torch.from_numpy(first + np.arange(len(data), dtype=np.int64)).to(device)
        buf[idx] = torch.from_numpy(data.copy()).to(device)
        planted = len(amps)
        del idx
    # soft-mask ~30% of 1 kbp blocks (case must be ignored by the scan)
    nb = (pos + 64) // 1024
    blk = buf[:nb * 1024].view(nb, 1024)
    mask = torch.rand(nb, generator=gen, device=device) < 0.3
    lower = blk[mask]
    is_upper = (lower >= 65) & (lower <= 90)
    blk[mask] = torch.where(is_upper, lower + 32, lower)
    return names, lens, buf, offs, planted


def plant_at_ends(buf, offs, lens, sts: STSSet, seed: int = 5, per_record: int = 3) -> int:
    """Overwrite the last bases of every record with `per_record` exact '+' amplicons of
    random STS: the last one ends on the record's final base, the others a few hundred
    bases before it.  Returns the number planted (plumbing for the record-end tests)."""
    import torch
    rng = np.random.default_rng(seed)
    n = 0
    for r, ln in enumerate(lens):
        end = int(ln)
        for _ in range(per_record):
            i = int(rng.integers(0, len(sts.ids)))
            a, b, size = sts.p1[i], sts.p2[i], int(sts.size[i])
            a, b = _concrete(rng, a), _concrete(rng, b)
            fill = _ACGT[rng.integers(0, 4, max(0, size - len(a) - len(b)))].tobytes()
            amp = a + fill + b
            start = end - len(amp)
            if start < 0:
                break
            o = int(offs[r]) + start
            buf[o:o + len(amp)] = torch.from_numpy(np.frombuffer(amp, dtype=np.uint8).copy()).to(buf.device)
            n += 1
            end = start - int(rng.integers(1, 200))
    return n
