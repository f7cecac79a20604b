"""Level-1 prefilter designs on c3's key set, simulated on the CPU.

Writes the pass rate (true-key windows included) of the product's blocked filter and of
alternatives over 20M uniform random 11-mer windows.  The keys come from the c3 table
(synth.make_sts(100000, W=11), the engine's sts_table keys): run with --make-keys first.
usage: python scripts/filter_sim.py [--make-keys]
"""
import sys
if "--make-keys" in sys.argv:
    import tempfile
    import numpy as np
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from merpcr_amd import MerPCR, synth
    sts = synth.make_sts(100000, W=11, iupac=0.0)
    fh = tempfile.NamedTemporaryFile("w", suffix=".sts", delete=False)
    fh.write(sts.text())
    fh.close()
    eng = MerPCR(wordsize=11, margin=50, mismatches=1)
    assert eng.load_sts_file(fh.name)
    np.save("/tmp/c3keys.npy", np.array(list(eng.sts_table.keys()), dtype=np.uint64))
import numpy as np
keys = np.load('/tmp/c3keys.npy').astype(np.uint64)
rng = np.random.default_rng(1)
win = rng.integers(0, 1 << 22, size=20_000_000, dtype=np.uint64)
keyset = np.zeros(1 << 22, dtype=bool); keyset[keys.astype(np.int64)] = True
true_rate = keyset[win.astype(np.int64)].mean()
print("keys", len(keys), "true-key window rate %.4f" % true_rate)

def blocked(words_log2, bitfuncs, word_fn, nwords=None):
    nw = nwords or (1 << words_log2)
    f = np.zeros(nw, dtype=np.uint64)
    wi = word_fn(keys)
    for bf in bitfuncs:
        np.bitwise_or.at(f, wi.astype(np.int64), (np.uint64(1) << bf(keys)))
    ww = word_fn(win)
    on = np.ones(len(win), dtype=bool)
    fw = f[ww.astype(np.int64)]
    for bf in bitfuncs:
        on &= ((fw >> bf(win)) & np.uint64(1)).astype(bool)
    return on.mean()

u = np.uint64
# current: 32-bit words, word = key bits 21..7, bits: 6..2 and 4..0
cur = blocked(15, [lambda k: (k >> u(2)) & u(31), lambda k: k & u(31)], lambda k: k >> u(7))
print("current 128KiB 2 bits/32b word: pass %.4f" % cur)
# k=1 direct top-20
print("k=1 direct 20 bits: pass %.4f" % blocked(15, [lambda k: (k >> u(2)) & u(31)], lambda k: k >> u(7)))
# independent second bit
h = lambda k: ((k * u(0x9E3779B1)) >> u(27)) & u(31)
print("2 bits, B hashed: %.4f" % blocked(15, [lambda k: (k >> u(2)) & u(31), h], lambda k: k >> u(7)))
# 64-bit blocks, 16K blocks (128 KiB): block = top 14 bits (21..8), k bits from 6-bit fields
for kk in (2, 3, 4):
    fs = [lambda k: (k >> u(2)) & u(63)]
    mults = [0x9E3779B1, 0x85EBCA6B, 0xC2B2AE35]
    for j in range(kk - 1):
        m = u(mults[j]); fs.append(lambda k, m=m: ((k * m) >> u(26)) & u(63))
    print("64b blocks k=%d: %.4f" % (kk, blocked(14, fs, lambda k: k >> u(8))))
# 32-bit words k=3
fs = [lambda k: (k >> u(2)) & u(31), lambda k: k & u(31), lambda k: ((k * u(0x85EBCA6B)) >> u(27)) & u(31)]
print("32b words k=3: %.4f" % blocked(15, fs, lambda k: k >> u(7)))
# 144 KiB: 36864 words, word = (key>>6 (16 bits) * 9) >> 4
wf = lambda k: ((k >> u(6)) * u(9)) >> u(4)
print("144KiB 2 bits: %.4f" % blocked(0, [lambda k: (k >> u(1)) & u(31), lambda k: ((k * u(0x9E3779B1)) >> u(27)) & u(31)], wf, nwords=36864))
# standard (unblocked) Bloom over 1M bits, k=2,3
for kk in (2, 3):
    f = np.zeros(1 << 20, dtype=bool)
    mults = [0x9E3779B1, 0x85EBCA6B, 0xC2B2AE35]
    for j in range(kk):
        f[((keys * u(mults[j])) >> u(12)) & u((1 << 20) - 1)] = True
    on = np.ones(len(win), dtype=bool)
    for j in range(kk):
        on &= f[(((win * u(mults[j])) >> u(12)) & u((1 << 20) - 1)).astype(np.int64)]
    print("unblocked Bloom 1M bits k=%d: %.4f" % (kk, on.mean()))
