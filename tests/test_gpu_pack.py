"""The device packer (pack_kernel, mp_genome.hip) against a numpy statement of the layout.

The planes are the coordinate system every hit is reported in (the reference walks the
upper-cased, FASTA-filtered sequence strings: src/merpcr/core/engine.py:373-411, 455;
src/merpcr/io/fasta.py:60).  Per base u = upper-case(byte) (a-z only):
  g2    2 bits, A=0 C=1 G=2 T=U=3, every other byte 0; base j of a word at bits 63-2j..62-2j
  ginv  1 bit (bit 63-j): u not in A/C/G/T/U
  gexc  1 bit: u not exactly A/C/G/T
  gwild 1 bit: u is 'N' (padding: 0)
  padding to 64 bases: code 0, ginv = gexc = 1
  run index: (global position, u) of every exception byte whose predecessor inside the
  same put is not the same exception character (sorted by position at seal).
Inputs cover every byte value, case, U, long runs across the kernel's 1 KiB pieces and
4 KiB tiles, ragged ends, chunked puts at offsets and unaligned device sources.
"""

import numpy as np
import pytest

from merpcr_amd import _native

pytestmark = pytest.mark.gpu


def _upper(b):
    u = b.copy()
    low = (u >= ord("a")) & (u <= ord("z"))
    u[low] -= 32
    return u


def _reference(seqs, puts):
    lens = [len(s) for s in seqs]
    base = np.concatenate([[0], np.cumsum([(n + 63) // 64 * 64 for n in lens])]).astype(np.int64)
    total = int(base[-1])
    code = np.zeros(total, dtype=np.uint64)
    exc = np.ones(total, dtype=bool)
    inv = np.ones(total, dtype=bool)
    wild = np.zeros(total, dtype=bool)
    runs = []
    for q, s in enumerate(seqs):
        u = _upper(s)
        c = np.zeros(len(u), dtype=np.uint64)
        for ch, v in ((b"A", 0), (b"C", 1), (b"G", 2), (b"T", 3), (b"U", 3)):
            c[u == ch[0]] = v
        acgt = np.isin(u, np.frombuffer(b"ACGT", dtype=np.uint8))
        acgtu = acgt | (u == ord("U"))
        b0 = int(base[q])
        code[b0:b0 + len(u)] = c
        exc[b0:b0 + len(u)] = ~acgt
        inv[b0:b0 + len(u)] = ~acgtu
        wild[b0:b0 + len(u)] = u == ord("N")
    for q, off, n in puts:
        u = _upper(seqs[q][off:off + n])
        e = ~np.isin(u, np.frombuffer(b"ACGT", dtype=np.uint8))
        head = e.copy()
        head[1:] &= ~(e[:-1] & (u[1:] == u[:-1]))
        for i in np.nonzero(head)[0]:
            runs.append((int(base[q]) + off + int(i), int(u[i])))
    runs.sort()
    sh = np.arange(62, -1, -2, dtype=np.uint64)
    g2 = np.bitwise_or.reduce(code.reshape(-1, 32) << sh, axis=1)
    bits = np.arange(63, -1, -1, dtype=np.uint64)
    ge = np.bitwise_or.reduce(exc.reshape(-1, 64).astype(np.uint64) << bits, axis=1)
    gi = np.bitwise_or.reduce(inv.reshape(-1, 64).astype(np.uint64) << bits, axis=1)
    gw = np.bitwise_or.reduce(wild.reshape(-1, 64).astype(np.uint64) << bits, axis=1)
    return g2, ge, gi, gw, runs


def _check(seqs, puts, device_src=False, misalign=0):
    import torch
    g = _native.Genome(0, [len(s) for s in seqs])
    stream = torch.cuda.current_stream().cuda_stream
    keep = []
    for q, off, n in puts:
        chunk = np.ascontiguousarray(seqs[q][off:off + n])
        if device_src:
            t = torch.zeros(n + misalign + 16, dtype=torch.uint8, device="cuda")
            t[misalign:misalign + n] = torch.from_numpy(chunk).cuda()
            keep.append(t)
            g.put_device(q, t.data_ptr() + misalign, n, offset=off, stream=stream)
        else:
            g.put(q, chunk, offset=off, stream=stream)
    g.seal(stream)
    torch.cuda.synchronize()
    g2, ge, gi, gw, xs, xc = g.download()
    g.close()
    r2, re_, ri, rw, runs = _reference(seqs, puts)
    assert np.array_equal(g2, r2), np.nonzero(g2 != r2)[0][:5]
    assert np.array_equal(ge, re_), np.nonzero(ge != re_)[0][:5]
    assert np.array_equal(gi, ri), np.nonzero(gi != ri)[0][:5]
    assert np.array_equal(gw, rw), np.nonzero(gw != rw)[0][:5]
    got = sorted(zip(xs.tolist(), xc.tolist()))
    assert got == runs, (len(got), len(runs), got[:5], runs[:5])


def _mixed(rng, n):
    """Mostly a/c/g/t of both cases with runs of one exception character (N, n, R, X, U, u,
    0xC5, 0x00, ...) of 1 - 5000 bytes, some starting on piece / tile boundaries."""
    s = np.frombuffer(b"ACGTacgt", dtype=np.uint8)[rng.integers(0, 8, n)].copy()
    pool = np.frombuffer(b"NnRXUuy-\xc5\x00\xff0", dtype=np.uint8)
    for _ in range(max(1, n // 3000)):
        ln = int(rng.integers(1, 5000))
        at = int(rng.integers(0, n)) if rng.random() < 0.7 else int(rng.integers(0, max(1, n // 1024))) * 1024
        s[at:at + ln] = pool[rng.integers(0, len(pool))]
    return s


def test_every_byte_value_single_put():
    rng = np.random.default_rng(5)
    s = rng.integers(0, 256, 100_003).astype(np.uint8)
    _check([s], [(0, 0, len(s))])


@pytest.mark.parametrize("device_src,misalign", [(False, 0), (True, 0), (True, 1), (True, 7)])
def test_chunked_puts_runs_across_tiles(device_src, misalign):
    rng = np.random.default_rng(11 + misalign)
    seqs = [_mixed(rng, n) for n in (70_000, 4096 * 3, 1, 63, 64, 65, 1024 * 5 + 17, 250_001)]
    puts = []
    for q, s in enumerate(seqs):
        off = 0
        while off < len(s):  # non-final chunks: multiples of 64
            n = min(len(s) - off, int(rng.integers(1, 40)) * 64 * int(rng.choice([1, 16, 64])))
            puts.append((q, off, n))
            off += n
    _check(seqs, puts, device_src=device_src, misalign=misalign)


def test_long_run_one_put():
    s = np.full(3 * 4096 + 100, ord("N"), dtype=np.uint8)
    s[:10] = ord("A")
    s[5000:5003] = ord("n")  # lower case: the same character after upper-casing
    s[-5:] = ord("g")
    _check([s], [(0, 0, len(s))])
