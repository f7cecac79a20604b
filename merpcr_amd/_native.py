"""ctypes binding of libmerpcr_hip.so (include/merpcr_hip.h).

The engine has no CPU fallback: if the library is missing, or no HIP device is
visible when a search runs, the calls raise.  Nothing here imports torch.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# MERPCR_LIB: an A/B variant library built in-tree (scripts/ablate.py, scripts/ab_lib.py)
LIB_PATH = os.environ.get("MERPCR_LIB") or os.path.join(_PKG, "_lib", "libmerpcr_hip.so")

MP_OK = 0
MP_E_ARG = -1
MP_E_HIP = -2
MP_E_NOMEM = -3
MP_E_STATE = -4
MP_E_CAP = -5
MP_E_IO = -6
MP_E_DECODE = -7
MP_STS_OK, MP_STS_BAD_LINE, MP_STS_PYTHON = 0, 1, 2

# every symbol include/merpcr_hip.h declares
EXPORTS = (
    "mp_abi_version", "mp_last_error", "mp_device_count",
    "mp_table_create", "mp_table_create_ex", "mp_table_stats", "mp_table_split", "mp_table_layout", "mp_table_destroy",
    "mp_genome_create", "mp_genome_put", "mp_genome_put_device", "mp_genome_seal",
    "mp_genome_stats", "mp_genome_download", "mp_genome_reset", "mp_genome_destroy",
    "mp_search_create", "mp_search_set_options", "mp_search_set_stage_timing", "mp_search_set_scan_timing", "mp_search_run",
    "mp_search_enqueue", "mp_search_complete", "mp_search_fetch", "mp_search_fetch_device", "mp_search_device_hits",
    "mp_search_last_stats", "mp_search_regrowths", "mp_search_dev_bytes", "mp_search_survivors", "mp_search_timing", "mp_search_destroy",
    "mp_multi_create", "mp_multi_genome", "mp_multi_put", "mp_multi_seal", "mp_multi_run", "mp_multi_fetch",
    "mp_multi_set_gather", "mp_multi_device_search", "mp_multi_timing", "mp_multi_destroy",
    "mp_comm_unique_id", "mp_comm_create", "mp_comm_gather_hits", "mp_comm_destroy",
    "mp_ipc_handle", "mp_ipc_open", "mp_ipc_close", "mp_search_put_hits",
    "mp_fasta_load", "mp_fasta_load_parallel", "mp_fasta_load_chunked", "mp_fasta_info", "mp_fasta_record_ascii", "mp_fasta_record", "mp_fasta_destroy",
    "mp_fasta_load_device", "mp_fasta_device_info", "mp_fasta_device_record", "mp_fasta_device_read",
    "mp_fasta_device_destroy",
    "mp_format_hits",
    "mp_sts_parse", "mp_sts_info", "mp_sts_arrays", "mp_sts_record_texts", "mp_sts_destroy",
)


class MPParams(ctypes.Structure):
    _fields_ = [("wordsize", c_int32), ("margin", c_int32), ("mismatches", c_int32),
                ("three_prime_match", c_int32), ("iupac_mode", c_int32)]


class MPRange(ctypes.Structure):
    _fields_ = [("seq_begin", c_uint32), ("seq_end", c_uint32),
                ("k_begin", c_uint64), ("k_end", c_uint64)]


MP_TAILS = {"auto": 0, "inline": 1, "kernel": 2}
MP_SORT = {"auto": 0, "radix64": 1, "radix128": 2, "scatter": 3}


class MPSearchOptions(ctypes.Structure):
    _fields_ = [("tails", c_int32), ("no_defer", c_int32), ("no_dense", c_int32), ("sort", c_int32),
                ("sort_bucket_bits", c_int32), ("pair_blocks_per_cu", c_int32),
                ("hit_cap", c_uint64), ("surv_cap", c_uint64), ("tail_cap", c_uint64),
                ("no_rank_filter", c_int32), ("no_split", c_int32),
                ("generic_forms", c_int32), ("ref32", c_int32), ("sched_short", c_int32), ("crowd_grid", c_int32),
                ("scan_grid", c_int32)]


class MPTableOptions(ctypes.Structure):
    _fields_ = [("lds_k", c_int32), ("no_h12", c_int32), ("kgrp4", c_int32), ("no_split", c_int32)]


ABI_VERSION = 3
MP_GENERIC = {"fix": 1, "gap": 2, "pair": 4}
MP_GATHER = {"copy": 0, "rccl": 1}


HIT_DTYPE = np.dtype([("pos1", "<u8"), ("pos2", "<u8"), ("seq", "<u4"), ("rec", "<u4")])


class NativeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libmerpcr_hip error {code}: {msg}")
        self.code = code


_lib = None


class _Tolerant:
    """A/B runs against older variant libraries (MERPCR_LIB): a symbol the library lacks
    takes its signature in a dummy, and calling it fails as a missing symbol would."""

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        try:
            return getattr(self._lib, name)
        except AttributeError:
            import types
            return types.SimpleNamespace()


def _sig(lib):
    if os.environ.get("MERPCR_LIB"):
        lib = _Tolerant(lib)
    P = c_void_p
    u64p = POINTER(c_uint64)
    lib.mp_abi_version.restype = c_int32
    lib.mp_last_error.restype = c_char_p
    lib.mp_device_count.argtypes = [POINTER(c_int32)]
    lib.mp_table_create.argtypes = [POINTER(MPParams), c_int32, c_uint32, P, P, P, P, P, P, P,
                                    POINTER(c_void_p)]
    lib.mp_table_create_ex.argtypes = [POINTER(MPParams), c_int32, c_uint32, P, P, P, P, P, P, P,
                                       POINTER(MPTableOptions), POINTER(c_void_p)]
    lib.mp_table_stats.argtypes = [P, u64p, u64p, u64p]
    lib.mp_table_split.argtypes = [P, POINTER(c_uint32), POINTER(c_uint32)]
    lib.mp_table_layout.argtypes = [P, POINTER(c_uint32)]
    lib.mp_table_destroy.argtypes = [P]
    lib.mp_table_destroy.restype = None
    lib.mp_genome_create.argtypes = [c_int32, c_uint32, P, POINTER(c_void_p)]
    lib.mp_genome_put.argtypes = [P, c_uint32, c_uint64, P, c_uint64, P]
    lib.mp_genome_put_device.argtypes = [P, c_uint32, c_uint64, P, c_uint64, P]
    lib.mp_genome_seal.argtypes = [P, P]
    lib.mp_genome_stats.argtypes = [P, u64p, u64p, u64p]
    lib.mp_genome_download.argtypes = [P, P, P, P, P, P, P]
    lib.mp_genome_reset.argtypes = [P, c_uint32, P]
    lib.mp_genome_destroy.argtypes = [P]
    lib.mp_genome_destroy.restype = None
    lib.mp_search_create.argtypes = [P, P, POINTER(c_void_p)]
    lib.mp_search_set_options.argtypes = [P, POINTER(MPSearchOptions)]
    lib.mp_search_set_stage_timing.argtypes = [P, c_int32]
    lib.mp_search_run.argtypes = [P, POINTER(MPRange), P, u64p]
    lib.mp_search_set_scan_timing.argtypes = [P, c_int32]
    lib.mp_search_enqueue.argtypes = [P, POINTER(MPRange), P]
    lib.mp_search_complete.argtypes = [P, u64p]
    lib.mp_search_regrowths.argtypes = [P, u64p]
    lib.mp_search_dev_bytes.argtypes = [P, u64p]
    lib.mp_search_fetch.argtypes = [P, P, c_uint64, P]
    lib.mp_search_fetch_device.argtypes = [P, P, c_uint64, P]
    lib.mp_search_device_hits.argtypes = [P, POINTER(c_void_p)]
    lib.mp_search_last_stats.argtypes = [P, POINTER(c_float), u64p, u64p]
    lib.mp_search_survivors.argtypes = [P, u64p]
    lib.mp_search_timing.argtypes = [P, POINTER(c_float), POINTER(c_float), POINTER(c_float), POINTER(c_float)]
    lib.mp_search_destroy.argtypes = [P]
    lib.mp_search_destroy.restype = None
    lib.mp_multi_create.argtypes = [c_uint32, POINTER(c_int32), POINTER(c_void_p), POINTER(c_void_p)]
    lib.mp_multi_genome.argtypes = [P, c_uint32, P]
    lib.mp_multi_put.argtypes = [P, c_uint32, P, c_uint64]
    lib.mp_multi_seal.argtypes = [P]
    lib.mp_multi_run.argtypes = [P, u64p]
    lib.mp_multi_set_gather.argtypes = [P, c_int32]
    lib.mp_multi_fetch.argtypes = [P, P, c_uint64]
    lib.mp_multi_device_search.argtypes = [P, c_uint32, POINTER(c_void_p), POINTER(MPRange), POINTER(c_float)]
    lib.mp_multi_timing.argtypes = [P, POINTER(c_float), POINTER(c_float)]
    lib.mp_multi_destroy.argtypes = [P]
    lib.mp_multi_destroy.restype = None
    lib.mp_comm_unique_id.argtypes = [P]
    lib.mp_comm_create.argtypes = [P, c_int32, c_int32, c_int32, POINTER(c_void_p)]
    lib.mp_comm_gather_hits.argtypes = [P, P, c_uint32, P, c_uint64, u64p, P]
    lib.mp_comm_destroy.argtypes = [P]
    lib.mp_comm_destroy.restype = None
    lib.mp_ipc_handle.argtypes = [P, P, u64p]
    lib.mp_ipc_open.argtypes = [P, c_int32, POINTER(c_void_p)]
    lib.mp_ipc_close.argtypes = [P]
    lib.mp_search_put_hits.argtypes = [P, P, c_uint64, P, u64p, P]
    lib.mp_fasta_load.argtypes = [c_char_p, POINTER(c_void_p)]
    lib.mp_fasta_load_chunked.argtypes = [c_char_p, c_uint64, POINTER(c_void_p)]
    lib.mp_fasta_load_parallel.argtypes = [c_char_p, c_int32, POINTER(c_void_p)]
    lib.mp_fasta_record_ascii.argtypes = [c_void_p, c_uint64, POINTER(c_int32)]
    lib.mp_fasta_info.argtypes = [P, u64p, u64p]
    lib.mp_fasta_record.argtypes = [P, c_uint64, POINTER(c_void_p), u64p, POINTER(c_void_p), u64p]
    lib.mp_fasta_destroy.argtypes = [P]
    lib.mp_fasta_destroy.restype = None
    lib.mp_fasta_load_device.argtypes = [c_char_p, c_int32, P, POINTER(c_void_p), POINTER(c_int32)]
    lib.mp_fasta_device_info.argtypes = [P, u64p, u64p, POINTER(c_void_p)]
    lib.mp_fasta_device_record.argtypes = [P, c_uint64, POINTER(c_void_p), u64p, u64p, u64p]
    lib.mp_fasta_device_read.argtypes = [P, c_uint64, c_uint64, P]
    lib.mp_fasta_device_destroy.argtypes = [P]
    lib.mp_fasta_device_destroy.restype = None
    lib.mp_sts_parse.argtypes = [c_char_p, c_int32, ctypes.c_int64, POINTER(c_void_p)]
    lib.mp_sts_info.argtypes = [P, POINTER(c_int32), u64p]
    lib.mp_sts_arrays.argtypes = [P, POINTER(c_void_p)]
    lib.mp_sts_record_texts.argtypes = [P, POINTER(c_void_p), POINTER(c_void_p), u64p]
    lib.mp_sts_destroy.argtypes = [P]
    lib.mp_sts_destroy.restype = None
    lib.mp_format_hits.argtypes = [P, c_uint64, P, P, c_uint32, P, P, c_uint32, P, c_uint64, u64p]


def _share_hip_runtime():
    """One HIP runtime per process.  A PyTorch-ROCm wheel bundles its own libamdhip64
    (soname libamdhip64.so.7, the same as /opt/rocm's), which libtorch_hip finds by file
    name.  If this library loaded /opt/rocm's copy first, a later `import torch` would map
    the second copy and its device init would fail ("No HIP GPUs are available").  So when
    torch is installed its runtime is mapped first (by path, RTLD_GLOBAL, without importing
    torch); libmerpcr_hip's NEEDED libamdhip64.so.7 then resolves to it, and torch later
    finds the same file already mapped."""
    import importlib.util
    if os.environ.get("MERPCR_SYSTEM_HIP") == "1":
        return
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
            return


def lib():
    """The loaded library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(the MI355X engine has no CPU fallback)")
        _share_hip_runtime()
        l = ctypes.CDLL(LIB_PATH)
        _sig(l)
        # MERPCR_LIB (A/B runs against an earlier build) admits the previous ABI as well
        if l.mp_abi_version() != ABI_VERSION and not (os.environ.get("MERPCR_LIB") and l.mp_abi_version() == 2):
            raise RuntimeError("libmerpcr_hip ABI version mismatch")
        _lib = l
    return _lib


def check(rc: int):
    if rc != MP_OK:
        msg = lib().mp_last_error().decode(errors="replace")
        if rc == MP_E_ARG:
            raise ValueError(msg)
        if rc == MP_E_IO:
            raise OSError(msg)
        raise NativeError(rc, msg)


def device_count() -> int:
    n = c_int32(0)
    check(lib().mp_device_count(ctypes.byref(n)))
    return n.value


def ptr(a: np.ndarray) -> c_void_p:
    return c_void_p(a.ctypes.data) if a.size else c_void_p(0)


class Table:
    """Device seed table (owns the native handle)."""

    def __init__(self, params: MPParams, device: int, key, hash_off, pcr_size, p1, p1_off, p2, p2_off,
                 lds_k: int = 0, h12: bool = True, kgrp4: str = "auto", split: bool = True):
        """Layout choices (mp_table_create_ex; the defaults are the library's own): lds_k 1..3 bits
        per key in the W 11..13 prefilter, h12 False keeps the 16-B IUPAC heads, kgrp4 "never" /
        "always" for the wide I = 1 key groups, split False keeps W 7..9 tables unsplit."""
        self._h = c_void_p()
        self.n_rec = len(key)
        key = np.ascontiguousarray(key, dtype=np.uint32)
        hash_off = np.ascontiguousarray(hash_off, dtype=np.uint32)
        pcr_size = np.ascontiguousarray(pcr_size, dtype=np.uint64)
        p1 = np.ascontiguousarray(p1, dtype=np.uint8)
        p2 = np.ascontiguousarray(p2, dtype=np.uint8)
        p1_off = np.ascontiguousarray(p1_off, dtype=np.uint64)
        p2_off = np.ascontiguousarray(p2_off, dtype=np.uint64)
        self.params = params
        opt = MPTableOptions(int(lds_k), 0 if h12 else 1, {"auto": 0, "never": 1, "always": -1}[kgrp4],
                             0 if split else 1)
        if not callable(lib().mp_table_create_ex):  # an ABI 2 library under MERPCR_LIB (A/B runs)
            check(lib().mp_table_create(ctypes.byref(params), device, self.n_rec, ptr(key), ptr(hash_off),
                                        ptr(pcr_size), ptr(p1), ptr(p1_off), ptr(p2), ptr(p2_off),
                                        ctypes.byref(self._h)))
            return
        check(lib().mp_table_create_ex(ctypes.byref(params), device, self.n_rec, ptr(key), ptr(hash_off),
                                       ptr(pcr_size), ptr(p1), ptr(p1_off), ptr(p2), ptr(p2_off),
                                       ctypes.byref(opt), ctypes.byref(self._h)))

    def stats(self):
        a, b, c = c_uint64(), c_uint64(), c_uint64()
        check(lib().mp_table_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"n_keys": a.value, "max_bucket": b.value, "dev_bytes": c.value}

    def split(self):
        """Split seeds (mp_table_split): {"seed_tables": 0/1/2, "rest_records": n}."""
        a, b = c_uint32(), c_uint32()
        check(lib().mp_table_split(self._h, ctypes.byref(a), ctypes.byref(b)))
        return {"seed_tables": a.value, "rest_records": b.value}

    LAYOUT = {"lds_exact": 1, "rank": 2, "kgrp": 4, "kgrp4": 8, "dense": 16, "split": 32, "hashed": 64,
              "defer_full": 128}

    def layout(self) -> set:
        """The seed structures the table holds (mp_table_layout), by name."""
        f = c_uint32()
        check(lib().mp_table_layout(self._h, ctypes.byref(f)))
        return {k for k, b in self.LAYOUT.items() if f.value & b}

    def close(self):
        if self._h:
            lib().mp_table_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Genome:
    """Sequences resident in HBM as 2-bit + exception planes."""

    def __init__(self, device: int, lengths):
        self._h = c_void_p()
        self.lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        check(lib().mp_genome_create(device, len(self.lengths), ptr(self.lengths), ctypes.byref(self._h)))

    def reset(self, lengths):
        """New sequence set on the same device buffers (grown only when needed)."""
        self.lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        check(lib().mp_genome_reset(self._h, len(self.lengths), ptr(self.lengths)))

    def put(self, seq: int, data: bytes, offset: int = 0, stream=None):
        buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        check(lib().mp_genome_put(self._h, seq, offset, ptr(buf), buf.size, c_void_p(stream or 0)))

    def put_device(self, seq: int, dev_ptr: int, nbytes: int, offset: int = 0, stream=None):
        check(lib().mp_genome_put_device(self._h, seq, offset, c_void_p(dev_ptr), nbytes, c_void_p(stream or 0)))

    def seal(self, stream=None):
        check(lib().mp_genome_seal(self._h, c_void_p(stream or 0)))

    def stats(self):
        a, b, c = c_uint64(), c_uint64(), c_uint64()
        check(lib().mp_genome_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return {"bases": a.value, "exc_runs": b.value, "dev_bytes": c.value}

    def download(self):
        """(g2, gexc, ginv, gwild, xr_start, xr_char) of the sealed genome (diagnostic, tests)."""
        total = int(sum((int(n) + 63) // 64 * 64 for n in self.lengths))
        n_xr = self.stats()["exc_runs"]
        g2 = np.empty(total // 32, dtype=np.uint64)
        ge = np.empty(total // 64, dtype=np.uint64)
        gi = np.empty(total // 64, dtype=np.uint64)
        gw = np.empty(total // 64, dtype=np.uint64)
        xs = np.empty(max(n_xr, 1), dtype=np.uint64)
        xc = np.empty(max(n_xr, 1), dtype=np.uint8)
        check(lib().mp_genome_download(self._h, ptr(g2), ptr(ge), ptr(gi), ptr(gw), ptr(xs), ptr(xc)))
        return g2, ge, gi, gw, xs[:n_xr], xc[:n_xr]

    def close(self):
        if self._h:
            lib().mp_genome_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Search:
    def __init__(self, table: Table, genome: Genome):
        self._h = c_void_p()
        self.table = table
        self.genome = genome
        check(lib().mp_search_create(table._h, genome._h, ctypes.byref(self._h)))

    def set_options(self, tails="auto", defer=True, dense=True, sort="auto", sort_bucket_bits=0,
                    pair_blocks_per_cu=0, hit_cap=0, surv_cap=0, tail_cap=0, rank_filter=True, split=True,
                    generic=(), ref32=False, sched_short=0, crowd_grid=0, scan_grid=0):
        """Kernel-path selection, initial list capacities and tuning (mp_search_set_options);
        the defaults are the library's automatic choices.  generic: names of MP_GENERIC ("fix",
        "gap", "pair": the run-time-shape kernel forms, for A/B runs)."""
        if isinstance(generic, str):
            generic = [g for g in generic.split("+") if g]
        gbits = 0
        for g in generic:
            gbits |= MP_GENERIC[g]
        o = MPSearchOptions(MP_TAILS[tails], 0 if defer else 1, 0 if dense else 1, MP_SORT[sort],
                            sort_bucket_bits, pair_blocks_per_cu, hit_cap, surv_cap, tail_cap,
                            0 if rank_filter else 1, 0 if split else 1, gbits, 1 if ref32 else 0,
                            int(sched_short), int(crowd_grid), int(scan_grid))
        check(lib().mp_search_set_options(self._h, ctypes.byref(o)))

    def set_stage_timing(self, on: bool):
        """Events around the tail, pair and order stages too (default on; off saves ~6 us
        per stage and run, and last_stats then reports those stages as -1)."""
        check(lib().mp_search_set_stage_timing(self._h, 1 if on else 0))

    def set_scan_timing(self, on: bool):
        """The scan kernel's own two events (default on; off, last_stats reports scan_ms -1)."""
        check(lib().mp_search_set_scan_timing(self._h, 1 if on else 0))

    def enqueue(self, rng=None, stream=None):
        """Enqueue a whole run on `stream` without waiting (mp_search_enqueue); complete()
        waits for it.  Lets the caller queue the next run (another handle) first."""
        r = MPRange(*rng) if rng is not None else None
        check(lib().mp_search_enqueue(self._h, ctypes.byref(r) if r is not None else None, c_void_p(stream or 0)))

    def complete(self) -> int:
        n = c_uint64(0)
        check(lib().mp_search_complete(self._h, ctypes.byref(n)))
        self._last_n = n.value
        return n.value

    def regrowths(self) -> int:
        n = c_uint64()
        check(lib().mp_search_regrowths(self._h, ctypes.byref(n)))
        return n.value

    def dev_bytes(self) -> int:
        """Device bytes of the handle's lists, sort buffers and order slots."""
        n = c_uint64()
        check(lib().mp_search_dev_bytes(self._h, ctypes.byref(n)))
        return n.value

    def run(self, rng=None, stream=None) -> int:
        n = c_uint64(0)
        r = None
        if rng is not None:
            r = MPRange(*rng)
        check(lib().mp_search_run(self._h, ctypes.byref(r) if r is not None else None,
                                  c_void_p(stream or 0), ctypes.byref(n)))
        self._last_n = n.value
        return n.value

    def last_hits(self) -> int:
        """Hits of this handle's last run (its own owned range)."""
        return getattr(self, "_last_n", 0)

    def fetch(self, n: int, stream=None) -> np.ndarray:
        out = np.empty(n, dtype=HIT_DTYPE)
        check(lib().mp_search_fetch(self._h, ptr(out), n, c_void_p(stream or 0)))
        return out

    def fetch_device(self, dev_ptr: int, cap: int, stream=None):
        """Copy the last run's hits into device memory at dev_ptr (cap entries)."""
        check(lib().mp_search_fetch_device(self._h, c_void_p(dev_ptr), cap, c_void_p(stream or 0)))

    def put_hits(self, dst: int, cap: int, count_dst: int, stream=None) -> int:
        """The last run's hits into dst (cap entries; another rank's buffer mapped by ipc_open
        on one node) and their count into the u64 at count_dst, by the copy engines on
        `stream` (mp_search_put_hits).  Returns the count; more than cap raises NativeError
        (code MP_E_CAP, nothing copied) whose ``need`` is the count."""
        n = c_uint64(0)
        rc = lib().mp_search_put_hits(self._h, c_void_p(dst), cap, c_void_p(count_dst), ctypes.byref(n),
                                      c_void_p(stream or 0))
        if rc == MP_E_CAP:
            e = NativeError(rc, lib().mp_last_error().decode(errors="replace"))
            e.need = n.value
            raise e
        check(rc)
        return n.value

    def device_hits(self) -> int:
        p = c_void_p()
        check(lib().mp_search_device_hits(self._h, ctypes.byref(p)))
        return p.value or 0

    def last_stats(self):
        ms, nw, nc = c_float(), c_uint64(), c_uint64()
        check(lib().mp_search_last_stats(self._h, ctypes.byref(ms), ctypes.byref(nw), ctypes.byref(nc)))
        sv = c_uint64()
        check(lib().mp_search_survivors(self._h, ctypes.byref(sv)))
        t1, t0, t2, t3 = c_float(), c_float(), c_float(), c_float()
        check(lib().mp_search_timing(self._h, ctypes.byref(t1), ctypes.byref(t0), ctypes.byref(t2), ctypes.byref(t3)))
        return {"scan_ms": ms.value, "windows": nw.value, "candidates": nc.value, "survivors": sv.value,
                "tail_ms": t0.value, "pair_ms": t2.value, "order_ms": t3.value}

    def close(self):
        if self._h:
            lib().mp_search_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Borrowed(Search):
    """A search handle owned by a Multi (stats only; never destroyed here)."""

    def __init__(self, h):
        self._h = h

    def close(self):
        self._h = c_void_p()


class Multi:
    """One process, several devices (mp_multi_*): owned ranges of one sequence set, one per
    device, searched in parallel and gathered into devices[0] by the copy engines (xGMI)."""

    def __init__(self, devices, tables):
        self.devices = [int(d) for d in devices]
        self.tables = list(tables)  # kept alive with the handle
        self._h = c_void_p()
        devs = (c_int32 * len(self.devices))(*self.devices)
        hs = (c_void_p * len(self.tables))(*[tb._h for tb in self.tables])
        check(lib().mp_multi_create(len(self.devices), devs, hs, ctypes.byref(self._h)))

    def genome(self, lengths):
        self.lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        check(lib().mp_multi_genome(self._h, len(self.lengths), ptr(self.lengths)))

    def put(self, seq: int, data):
        buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data,
                                   dtype=np.uint8)
        check(lib().mp_multi_put(self._h, seq, ptr(buf), buf.size))

    def seal(self):
        check(lib().mp_multi_seal(self._h))

    def set_gather(self, mode: str):
        """"copy" (default: peer copies by the copy engines) or "rccl" (distinct devices)."""
        check(lib().mp_multi_set_gather(self._h, MP_GATHER[mode]))

    def run(self) -> int:
        n = c_uint64(0)
        check(lib().mp_multi_run(self._h, ctypes.byref(n)))
        return n.value

    def fetch(self, n: int) -> np.ndarray:
        out = np.empty(n, dtype=HIT_DTYPE)
        check(lib().mp_multi_fetch(self._h, ptr(out), n))
        return out

    def device(self, i: int):
        """(search handle of device i, its owned range, last gather ms)."""
        s, r, g = c_void_p(), MPRange(), c_float()
        check(lib().mp_multi_device_search(self._h, i, ctypes.byref(s), ctypes.byref(r), ctypes.byref(g)))
        return _Borrowed(s), (r.seq_begin, r.seq_end, r.k_begin, r.k_end), g.value

    def timing(self):
        """(span_ms, gather_ms) of the last run on devices[0]'s stream."""
        sp, g = c_float(), c_float()
        check(lib().mp_multi_timing(self._h, ctypes.byref(sp), ctypes.byref(g)))
        return sp.value, g.value

    def close(self):
        if self._h:
            lib().mp_multi_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


IPC_HANDLE_BYTES = 64


def ipc_handle(dev_ptr: int):
    """Export the device allocation holding dev_ptr to the other processes of the node
    (mp_ipc_handle): (handle bytes, dev_ptr's offset in the allocation)."""
    buf = (ctypes.c_uint8 * IPC_HANDLE_BYTES)()
    off = c_uint64(0)
    check(lib().mp_ipc_handle(c_void_p(dev_ptr), buf, ctypes.byref(off)))
    return bytes(buf), off.value


def ipc_open(handle: bytes, device: int) -> int:
    """Map another process's exported allocation on `device`; returns its base address here
    (add the exporter's offset)."""
    b = (ctypes.c_uint8 * IPC_HANDLE_BYTES).from_buffer_copy(handle)
    p = c_void_p()
    check(lib().mp_ipc_open(b, device, ctypes.byref(p)))
    return p.value or 0


def ipc_close(dev_ptr: int):
    check(lib().mp_ipc_close(c_void_p(dev_ptr)))


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    check(lib().mp_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """One rank of a process-per-GPU job (mp_comm_*): RCCL inside the library; the
    128-byte unique id is shared by the caller (e.g. over torch.distributed)."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int):
        self._h = c_void_p()
        self.rank, self.nranks = rank, nranks
        b = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().mp_comm_create(b, nranks, rank, device, ctypes.byref(self._h)))

    def gather_hits(self, search: Search, dev_out: int, cap: int, seq_shift: int = 0, stream=None) -> int:
        """Every rank's last-run hits into dev_out on rank 0, rank order; returns the total."""
        n = c_uint64(0)
        rc = lib().mp_comm_gather_hits(self._h, search._h, seq_shift, c_void_p(dev_out), cap, ctypes.byref(n),
                                       c_void_p(stream or 0))
        self.last_total = n.value  # set on MP_E_CAP too: the capacity rank 0 needs
        check(rc)
        return n.value

    def close(self):
        if self._h:
            lib().mp_comm_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _decode_error(rc):
    if rc == MP_E_DECODE:
        msg = lib().mp_last_error().decode(errors="replace")
        pos = int(msg.rsplit(" ", 1)[-1])
        raise UnicodeDecodeError("utf-8", b"", pos, pos + 1, msg)


def sts_parse(path: str, wordsize: int, default_pcr_size: int):
    """Parse an STS file natively (mp_sts_parse).  Returns a dict of numpy arrays and
    counters (copies; the native handle is released)."""
    h = c_void_p()
    rc = lib().mp_sts_parse(os.fsencode(path), wordsize, default_pcr_size, ctypes.byref(h))
    _decode_error(rc)
    check(rc)
    try:
        st = c_int32()
        cnt = (c_uint64 * 10)()
        check(lib().mp_sts_info(h, ctypes.byref(st), cnt))
        n, nt = cnt[0], cnt[9]
        ptrs = (c_void_p * 12)()
        check(lib().mp_sts_arrays(h, ptrs))

        def arr(i, dtype, count):
            if not count:
                return np.zeros(0, dtype=dtype)
            return np.ctypeslib.as_array(ctypes.cast(ptrs[i], POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                         shape=(count,)).copy()

        tp, op, nb = c_void_p(), c_void_p(), c_uint64()
        check(lib().mp_sts_record_texts(h, ctypes.byref(tp), ctypes.byref(op), ctypes.byref(nb)))
        rec_text = (np.ctypeslib.as_array(ctypes.cast(tp, POINTER(ctypes.c_uint8)), shape=(nb.value,)).copy()
                    if nb.value else np.zeros(0, dtype=np.uint8))
        rec_off = np.ctypeslib.as_array(ctypes.cast(op, POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy()
        return {"status": st.value, "n": n, "bad_line": cnt[1], "short": cnt[2], "ambig": cnt[3],
                "rec_text": rec_text, "rec_text_off": rec_off,
                "badsize": cnt[4], "max_pcr_size": cnt[5],
                "key": arr(0, np.uint32, n), "hash_off": arr(1, np.uint32, n), "pcr_size": arr(2, np.uint64, n),
                "line": arr(3, np.uint64, n), "direct": arr(4, np.uint8, n), "text_idx": arr(5, np.uint32, n),
                "p1": arr(6, np.uint8, cnt[6]), "p1_off": arr(7, np.uint64, n + 1),
                "p2": arr(8, np.uint8, cnt[7]), "p2_off": arr(9, np.uint64, n + 1),
                "text": arr(10, np.uint8, cnt[8]), "text_off": arr(11, np.uint64, nt + 1)}
    finally:
        lib().mp_sts_destroy(h)


def fasta_read(path: str, chunk_bytes: int = 0, threads: int = 0, with_ascii: bool = False):
    """Read a FASTA file natively; returns [(defline, sequence bytes)].

    Raises UnicodeDecodeError for invalid UTF-8, as the reference's text-mode read does.
    Default: the parallel whole-file reader (mp_fasta_load_parallel, `threads` host threads,
    0 = every usable CPU).  chunk_bytes > 0 (tests): the streaming reader with that read size.
    Sequences are views of the reader's buffers (freed with the last view); with_ascii adds
    each record's "ASCII only" flag as a third field.
    """
    h = c_void_p()
    if chunk_bytes:
        rc = lib().mp_fasta_load_chunked(os.fsencode(path), chunk_bytes, ctypes.byref(h))
    else:
        rc = lib().mp_fasta_load_parallel(os.fsencode(path), threads, ctypes.byref(h))
    _decode_error(rc)
    check(rc)
    owner = _FastaHandle(h)
    n, total = c_uint64(), c_uint64()
    check(lib().mp_fasta_info(h, ctypes.byref(n), ctypes.byref(total)))
    out = []
    dp, dl, sp, sl = c_void_p(), c_uint64(), c_void_p(), c_uint64()
    for i in range(n.value):
        check(lib().mp_fasta_record(h, i, ctypes.byref(dp), ctypes.byref(dl), ctypes.byref(sp), ctypes.byref(sl)))
        d = ctypes.string_at(dp, dl.value).decode("utf-8")
        if sl.value:  # the reader's buffer itself (no copy); the view keeps the handle alive
            arr = (ctypes.c_uint8 * sl.value).from_address(sp.value)
            arr._owner = owner
            seq = memoryview(arr).cast("B")
        else:
            seq = b""
        if with_ascii:
            asc = c_int32()
            check(lib().mp_fasta_record_ascii(h, i, ctypes.byref(asc)))
            out.append((d, seq, bool(asc.value)))
        else:
            out.append((d, seq))
    return out


class _FastaHandle:
    """Owns an mp_fasta handle; record views made by fasta_read reference it."""

    def __init__(self, h):
        self._h = h

    def __del__(self):
        try:
            if self._h:
                lib().mp_fasta_destroy(self._h)
                self._h = None
        except Exception:
            pass


class _FastaDeviceHandle:
    """Owner of a device-ingested FASTA (mp_fasta_load_device): its filtered bases stay in
    device memory until the last DeviceSpan over them is gone."""

    def __init__(self, h, device: int):
        self._h = h
        self.device = device

    def read(self, offset: int, n: int) -> bytes:
        out = np.empty(n, dtype=np.uint8)
        if n:
            check(lib().mp_fasta_device_read(self._h, offset, n, ptr(out)))
        return out.tobytes()

    def __del__(self):
        try:
            if self._h:
                lib().mp_fasta_device_destroy(self._h)
                self._h = None
        except Exception:
            pass


class DeviceSpan:
    """n bases of a device-ingested FASTA at device address ptr (device `device`): what
    mp_genome_put_device packs without a host copy.  Slices are spans; host() copies."""

    __slots__ = ("owner", "offset", "n", "base")

    def __init__(self, owner: _FastaDeviceHandle, base: int, offset: int, n: int):
        self.owner, self.base, self.offset, self.n = owner, base, offset, n

    @property
    def device(self) -> int:
        return self.owner.device

    @property
    def ptr(self) -> int:
        return self.base + self.offset

    def __len__(self):
        return self.n

    def __getitem__(self, sl):
        start, stop, step = sl.indices(self.n)
        assert step == 1, "contiguous slices only"
        return DeviceSpan(self.owner, self.base, self.offset + start, max(0, stop - start))

    def host(self) -> bytes:
        return self.owner.read(self.offset, self.n)


def fasta_read_device(path: str, device: int, stream=None):
    """[(defline, DeviceSpan)] of an ASCII FASTA file ingested on `device`
    (mp_fasta_load_device), or None when the file needs the host reader (a byte >= 0x80)."""
    h, asc = c_void_p(), c_int32()
    check(lib().mp_fasta_load_device(os.fsencode(path), device, c_void_p(stream or 0), ctypes.byref(h),
                                     ctypes.byref(asc)))
    if not asc.value:
        return None
    if not h.value:  # an empty file or one without a header line: no record
        return []
    owner = _FastaDeviceHandle(h, device)
    n, total, base = c_uint64(), c_uint64(), c_void_p()
    check(lib().mp_fasta_device_info(h, ctypes.byref(n), ctypes.byref(total), ctypes.byref(base)))
    out = []
    dp, dl, off, ln = c_void_p(), c_uint64(), c_uint64(), c_uint64()
    for i in range(n.value):
        check(lib().mp_fasta_device_record(h, i, ctypes.byref(dp), ctypes.byref(dl), ctypes.byref(off), ctypes.byref(ln)))
        out.append((ctypes.string_at(dp, dl.value).decode("ascii"), DeviceSpan(owner, base.value or 0, off.value, ln.value)))
    return out


def _csr(items):
    """UTF-8 bytes of each string, concatenated, with offsets."""
    enc = [x.encode("utf-8") for x in items]
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    if enc:
        np.cumsum([len(b) for b in enc], out=off[1:])
    return np.frombuffer(b"".join(enc), dtype=np.uint8), off


class Formatter:
    """Output-line formatter over fixed label and record texts (mp_format_hits)."""

    def __init__(self, labels, rec_texts, rec_off=None):
        """rec_texts: one str per record, or (rec_off given) their UTF-8 bytes concatenated
        as a uint8 array with len + 1 offsets."""
        self.labels, self.label_off = _csr(labels)
        if rec_off is None:
            self.rec, self.rec_off = _csr(rec_texts)
        else:
            self.rec = np.ascontiguousarray(rec_texts, dtype=np.uint8)
            self.rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
        self.n_seq, self.n_rec = len(labels), len(self.rec_off) - 1

    def __call__(self, hits: np.ndarray) -> bytes:
        hits = np.ascontiguousarray(hits, dtype=HIT_DTYPE)
        n = c_uint64()
        args = (ptr(hits), hits.size, ptr(self.labels), ptr(self.label_off), self.n_seq,
                ptr(self.rec), ptr(self.rec_off), self.n_rec)
        check(lib().mp_format_hits(*args, None, 0, ctypes.byref(n)))
        out = np.empty(n.value, dtype=np.uint8)
        check(lib().mp_format_hits(*args, ptr(out), out.size, ctypes.byref(n)))
        return out.tobytes()
