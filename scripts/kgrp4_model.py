"""Model of the key references c4's wide key groups (kgrp4) leave for tail_kernel, per field
layout: every 32-key group of the table, each present key's pass rate
for a uniform random window (N mismatches over its field's plain bases; keys without a field
pass), times 3e9 / 4^W windows.  CPU only.  usage: python scripts/kgrp4_model.py"""
import collections
import math
import os
import sys
import tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from merpcr_amd import synth, MerPCR
cfg = synth.CONFIGS['c4']
sts = synth.make_sts(cfg['n_sts'], W=cfg['W'], iupac=cfg['iupac'])
eng = MerPCR(wordsize=cfg['W'], margin=cfg['M'], mismatches=cfg['N'], iupac_mode=cfg['I'])
with tempfile.NamedTemporaryFile('w', suffix='.sts', delete=False) as fh:
    fh.write(sts.text())
eng.load_sts_file(fh.name)
W, N = cfg['W'], cfg['N']
recs = eng._recs
keys = eng._record_keys(recs)
buck = collections.defaultdict(list)
for r, k in zip(recs, keys):
    buck[int(k)].append(r)
print('records', len(recs), 'keys', len(buck))
def pr(p):  # pass rate of p plain bases at N mismatches, random window bases
    return sum(math.comb(p, m) * 3**m for m in range(N + 1) if m <= p) / 4**p
def plain_count(r, F):
    if r.hash_offset != 0: return None
    p1 = r.primer1.upper()
    if len(p1) <= W or any(c not in 'ACGT' for c in p1[:W]): return None
    return sum(1 for c in p1[W:W+F] if c in 'ACGT')
groups = collections.defaultdict(list)
for k in sorted(buck): groups[k >> 5].append(k)
def refs(fmt):
    tot = 0.0; parts = collections.Counter()
    for g, ks in groups.items():
        n = len(ks)
        slots = fmt(n)  # list of F per field slot
        for j, k in enumerate(ks):
            b = buck[k]
            if j >= len(slots): tot += 1; parts['no slot'] += 1; continue
            if len(b) != 1: tot += 1; parts['multi'] += 1; continue
            p = plain_count(b[0], slots[j])
            if p is None: tot += 1; parts['nofield'] += 1; continue
            tot += pr(p); parts['field'] += pr(p)
    f = 3e9 / 4**W
    return tot * f / 1e6, {k: round(v * f / 1e6, 2) for k, v in parts.items()}
print('current 3x10', refs(lambda n: [10, 10, 10]))
print('adaptive 3x10/4x8/5x6', refs(lambda n: [10]*3 if n <= 3 else ([8]*4 if n == 4 else [6]*5)))
print('adaptive 3x10/4x8', refs(lambda n: [10]*3 if n <= 3 else [8]*4))
hist = collections.Counter(len(v) for v in buck.values()); print('bucket sizes', sorted(hist.items())[:8])
gh = collections.Counter(len(v) for v in groups.values()); print('group sizes', sorted(gh.items()))
L = collections.Counter(len(r.primer1) for r in recs); print('primer1 len', sorted(L.items()))
P = collections.Counter(plain_count(r, 10) for r in recs); print('plain of 10', sorted(P.items(), key=lambda x: (x[0] is None, x[0])))
def refs2():
    tot = collections.Counter()
    for g, ks in groups.items():
        n = len(ks)
        if n >= 4:
            for j, k in enumerate(ks):
                b = buck[k]
                if j >= 4 or len(b) != 1: tot['noslot/multi'] += 1; continue
                p = plain_count(b[0], 8)
                if p is None: tot['nofield'] += 1; continue
                tot['field8'] += pr(p)
            continue
        s = 0
        for j, k in enumerate(ks):
            b = buck[k]
            need = len(b)
            if s + need > 3 or need > 2:
                tot['noslot'] += 1; s += 1; continue  # no room: presence alone (keeps one slot empty)
            ps = [plain_count(r, 10) for r in b]
            if any(p is None for p in ps): tot['nofield'] += 1; s += need; continue
            tot['field10' if need == 1 else 'pair'] += sum(pr(p) for p in ps)
            s += need
    f = 3e9 / 4**W
    return round(sum(tot.values()) * f / 1e6, 2), {k: round(v * f / 1e6, 2) for k, v in tot.items()}
print('3x10 with pairs / 4x8', refs2())
def refs3(pairs):
    tot = collections.Counter()
    for g, ks in groups.items():
        np_ = len(ks)
        used2 = False
        for j, k in enumerate(ks):
            b = buck[k]
            if j >= 4 or (j == 3 and np_ < 4): tot['noslot'] += 1; continue
            F = 6 if j == 3 else (8 if np_ >= 4 else 10)
            if len(b) == 2 and pairs and np_ <= 2 and not used2 and j < 2:
                ps = [plain_count(r, 10) for r in b]
                if all(p is not None for p in ps):
                    used2 = True; tot['pair'] += min(1, pr(ps[0]) + pr(ps[1])); continue
            if len(b) != 1: tot['multi'] += 1; continue
            p = plain_count(b[0], F)
            if p is None: tot['nofield'] += 1; continue
            tot['field%d' % F] += pr(p)
    f = 3e9 / 4**W
    return round(sum(tot.values()) * f / 1e6, 2), {k: round(v * f / 1e6, 2) for k, v in tot.items()}
print('A 3x10 + 4th 6-base spare', refs3(False))
print('B A + pairs in slot 2', refs3(True))
