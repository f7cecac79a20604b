"""Native hit formatter (mp_format_hits) vs the reference's print line.

Expected lines are the f-string of src/merpcr/core/engine.py:442, built here in
Python from the same hits; the native side is what MerPCR.search writes.
"""

import os

import numpy as np
import pytest

from merpcr_amd import _native

pytestmark = pytest.mark.skipif(not os.path.exists(_native.LIB_PATH), reason="library not built")

LABELS = ["chr1", "L78833", "séq_ſ", "x" * 300, "中文"]
RECS = [("AFM248yg9", "(D17S932)  Chr.17, 63.7 cM", "-"), ("s1", "", "+"), ("é", "a\x0bb\x1cc", "+"),
        ("id", "alias with spaces", "-")]


def _expected(hits):
    out = []
    for p1, p2, sq, ri in zip(hits["pos1"].tolist(), hits["pos2"].tolist(), hits["seq"].tolist(),
                              hits["rec"].tolist()):
        i, a, d = RECS[ri]
        out.append(f"{LABELS[sq]}\t{p1 + 1}..{p2 + 1}\t{i}\t{a}\t({d})\n")
    return "".join(out).encode("utf-8")


def _hits(n, seed):
    rng = np.random.default_rng(seed)
    h = np.zeros(n, dtype=_native.HIT_DTYPE)
    p1 = rng.integers(0, 1 << 40, n, dtype=np.uint64)
    p1[: min(n, 4)] = [0, 8, 9, 99][: min(n, 4)]
    h["pos1"] = p1
    h["pos2"] = p1 + rng.integers(0, 20000, n, dtype=np.uint64)
    h["seq"] = rng.integers(0, len(LABELS), n)
    h["rec"] = rng.integers(0, len(RECS), n)
    return h


def _fmt():
    return _native.Formatter(LABELS, [f"{i}\t{a}\t({d})" for i, a, d in RECS])


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 300_000])
def test_format_matches_print(n):
    h = _hits(n, n)
    assert _fmt()(h) == _expected(h)


def test_format_edge_coordinates():
    h = np.zeros(3, dtype=_native.HIT_DTYPE)
    h["pos1"] = [0, 2**64 - 2, 999_999_999]
    h["pos2"] = [0, 2**64 - 2, 1_000_000_000]
    assert _fmt()(h) == _expected(h)


def test_format_rejects_bad_indices():
    h = _hits(3, 1)
    h["rec"][2] = len(RECS)
    with pytest.raises(ValueError):
        _fmt()(h)
    h = _hits(3, 1)
    h["seq"][0] = len(LABELS)
    with pytest.raises(ValueError):
        _fmt()(h)
