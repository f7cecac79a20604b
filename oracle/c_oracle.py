"""ctypes wrapper of the C oracle (oracle/epcr_oracle.c).  TEST INFRASTRUCTURE ONLY.

The records, keys and hash offsets come from the Python oracle's own STS loader
(oracle/epcr_oracle.py), so nothing of the product path is involved.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_int32, c_int64, c_uint32, c_void_p

import numpy as np

from . import epcr_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libepcr_oracle.so")
HIT_DTYPE = np.dtype([("pos1", "<u8"), ("pos2", "<u8"), ("seq", "<u4"), ("rec", "<u4")])


class _Params(ctypes.Structure):
    _fields_ = [("W", c_int32), ("M", c_int32), ("N", c_int32), ("X", c_int32), ("I", c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        l = ctypes.CDLL(LIB)
        l.oracle_search.restype = c_int64
        l.oracle_search.argtypes = [POINTER(_Params), c_uint32, c_void_p, c_void_p, c_uint32, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                    POINTER(c_void_p)]
        l.oracle_free.argtypes = [c_void_p]
        l.oracle_free.restype = None
        _lib = l
    return _lib


def _ptr(a):
    return c_void_p(a.ctypes.data) if a.size else c_void_p(0)


def table_arrays(table: O.OracleTable):
    recs = table.records
    enc = lambda s: s.encode("latin-1", errors="replace")  # primers in the fixtures are ASCII
    key = np.array([r.key for r in recs], dtype=np.uint32)
    off = np.array([r.hash_offset for r in recs], dtype=np.uint32)
    size = np.array([r.pcr_size for r in recs], dtype=np.uint64)
    b1 = [enc(r.primer1) for r in recs]
    b2 = [enc(r.primer2) for r in recs]
    o1 = np.zeros(len(recs) + 1, dtype=np.uint64)
    o2 = np.zeros(len(recs) + 1, dtype=np.uint64)
    if recs:
        o1[1:] = np.cumsum([len(b) for b in b1])
        o2[1:] = np.cumsum([len(b) for b in b2])
    return (key, off, size, np.frombuffer(b"".join(b1) or b"\0", dtype=np.uint8), o1,
            np.frombuffer(b"".join(b2) or b"\0", dtype=np.uint8), o2)


def search(table: O.OracleTable, seqs, p: dict, nthreads: int = 1) -> np.ndarray:
    """Hits (pos1, pos2, seq, rec) of byte sequences in the reference's order."""
    arrs = [np.ascontiguousarray(np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray))
                                 else s, dtype=np.uint8) for s in seqs]
    ptrs = (c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
    lens = np.array([a.size for a in arrs], dtype=np.uint64)
    key, off, size, b1, o1, b2, o2 = table_arrays(table)
    prm = _Params(p["wordsize"], p["margin"], p["mismatches"], p["three_prime_match"], p["iupac_mode"])
    out = c_void_p()
    n = lib().oracle_search(ctypes.byref(prm), len(arrs), ptrs, _ptr(lens), len(table.records), _ptr(key),
                            _ptr(off), _ptr(size), _ptr(b1), _ptr(o1), _ptr(b2), _ptr(o2), nthreads,
                            ctypes.byref(out))
    if n < 0:
        raise MemoryError("oracle_search failed")
    res = np.empty(n, dtype=HIT_DTYPE)
    if n:
        ctypes.memmove(res.ctypes.data, out.value, n * HIT_DTYPE.itemsize)
    lib().oracle_free(out)
    return res


def lines(table: O.OracleTable, records, p: dict, nthreads: int = 1):
    """Output lines for (label, sequence-str) records, as the reference prints them."""
    hits = search(table, [s.upper().encode("latin-1", errors="replace") if not s.isascii() else s.encode()
                          for _, s in records], p, nthreads)
    out = []
    for h in hits:
        r = table.records[int(h["rec"])]
        out.append(f"{records[int(h['seq'])][0]}\t{int(h['pos1']) + 1}..{int(h['pos2']) + 1}\t{r.sts_id}\t"
                   f"{r.alias}\t({r.direct})")
    return out
