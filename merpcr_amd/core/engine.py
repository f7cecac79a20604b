"""MerPCR -- drop-in search engine whose hot path runs on MI355X.

Same constructor, attributes and methods as the reference class
(src/merpcr/core/engine.py:44-642).  ``load_sts_file`` and the primer helpers
are host-side bookkeeping with the reference's exact semantics; ``search``
hands the seed table and the sequences to libmerpcr_hip.so (HIP kernels on the
GPU) and only formats the sorted hits it gets back.  There is no CPU search
path: without the library or a HIP device, ``search`` raises.

Output order and content follow the reference's single-chunk (``-T 1``)
semantics for every record; see DESIGN.md ("Threads") for the documented
difference from the reference's multi-process chunking when threads > 1.
"""

from __future__ import annotations

import logging
import os
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..io.fasta import FASTALoader, _utf8_locale
from .encode import CharCodes
from .models import FASTARecord, STSHit, STSRecord, ThreadData

AMBIG = 100
MIN_FILESIZE_FOR_THREADING = 100000

DEFAULT_MARGIN = 50
DEFAULT_WORDSIZE = 11
DEFAULT_MISMATCHES = 0
DEFAULT_THREE_PRIME_MATCH = 1
DEFAULT_IUPAC_MODE = 0
DEFAULT_THREADS = 1
DEFAULT_PCR_SIZE = 240

MIN_WORDSIZE = 3
MAX_WORDSIZE = 16
MIN_MISMATCHES = 0
MAX_MISMATCHES = 10
MIN_MARGIN = 0
MAX_MARGIN = 10000
MIN_THREE_PRIME_MATCH = 0
MIN_PCR_SIZE = 1
MAX_PCR_SIZE = 10000

# the reference's module logger name (src/merpcr/core/engine.py: getLogger(__name__)), so
# that code configuring the "merpcr" logger hierarchy sees this engine's messages too
logger = logging.getLogger("merpcr.core.engine")

_CODE2 = {"A": 0, "C": 1, "G": 2, "T": 3, "U": 3}
_COMPL_BASE = {"A": "T", "C": "G", "G": "C", "T": "A", "U": "A", "B": "V", "D": "H",
               "H": "D", "K": "M", "M": "K", "N": "N", "R": "Y", "S": "S", "V": "B",
               "W": "W", "X": "X", "Y": "R"}
_IUPAC_SETS = {"A": "A", "C": "C", "G": "G", "T": "TU", "U": "TU", "R": "AGR", "Y": "CTUY",
               "M": "ACM", "K": "GTUK", "S": "CGS", "W": "ATUW", "B": "CGTUYKSB",
               "D": "AGTURKWD", "H": "ACTUYMWH", "V": "ACGRMSV", "N": "ACGTURYMKSWBDHVN"}


class _LazyRecords(list):
    """``sts_records`` of a natively parsed STS file: a real list (the reference's
    ``List[STSRecord]``, engine.py:62) whose STSRecord objects are built from the parser's
    arrays on first use -- any read or write of the list.  The device search, the table
    build and the formatter read the arrays and never touch it, so a CLI run builds no
    record object (200k of them took 0.6 s for 100k STS)."""

    __slots__ = ("_src", "_n", "_mutated")

    def __init__(self, src, n: int):
        super().__init__()
        self._src = src  # _NativeRecords, shared with the table view; None once built
        self._n = n
        self._mutated = False

    def _ready(self):
        if self._src is not None:
            src, self._src = self._src, None
            src.materialize()

    def native_len(self):
        """Record count without building the records (None after a mutation)."""
        if self._src is not None:
            return self._n
        return None if self._mutated else list.__len__(self)

    def __reduce__(self):  # pickles as the plain list
        self._ready()
        return (list, (list(list.__iter__(self)),))


class _LazyTable(dict):
    """``sts_table`` of a natively parsed STS file: a real dict (engine.py:63) of key ->
    bucket list, holding the same record objects as ``sts_records``, filled on first use."""

    __slots__ = ("_src",)

    def __init__(self, src):
        super().__init__()
        self._src = src

    def _ready(self):
        if self._src is not None:
            src, self._src = self._src, None
            src.materialize()

    def __reduce__(self):
        self._ready()
        return (dict, (dict(dict.items(self)),))


def _wrap(cls, base, names, mutating):
    for name in names:
        fn = getattr(base, name)

        def method(self, *a, __fn=fn, **k):
            self._ready()
            if mutating and hasattr(self, "_mutated"):
                self._mutated = True
            return __fn(self, *a, **k)

        method.__name__ = name
        setattr(cls, name, method)


_wrap(_LazyRecords, list, ("__len__", "__getitem__", "__iter__", "__reversed__", "__contains__", "__eq__",
                           "__ne__", "__lt__", "__le__", "__gt__", "__ge__", "__add__", "__mul__", "__rmul__",
                           "__repr__", "index", "count", "copy"), False)
_wrap(_LazyRecords, list, ("__setitem__", "__delitem__", "__iadd__", "__imul__", "append", "extend", "insert",
                           "pop", "remove", "sort", "reverse", "clear"), True)
_wrap(_LazyTable, dict, ("__len__", "__getitem__", "__iter__", "__reversed__", "__contains__", "__eq__", "__ne__",
                         "__repr__", "__or__", "__ror__", "get", "keys", "values", "items", "copy",
                         "__setitem__", "__delitem__", "__ior__", "setdefault", "pop", "popitem", "update",
                         "clear"), False)


class _NativeRecords:
    """The parser's arrays behind a lazy ``sts_records`` / ``sts_table`` pair; builds the
    STSRecord objects (and the buckets, in file order) once, into both containers."""

    def __init__(self, r):
        self.r = r
        self.recs = None
        self.table = None
        self._blob = None

    def materialize(self):
        r, recs, table = self.r, self.recs, self.table
        if r is None:
            return
        self.r = None
        p1s = r["p1"].tobytes().decode("ascii")
        p2s = r["p2"].tobytes().decode("ascii")
        p1o, p2o = r["p1_off"].tolist(), r["p2_off"].tolist()
        text, to = r["text"].tobytes(), r["text_off"].tolist()
        if text.isascii():
            ts = text.decode("ascii")
            items = [ts[to[i]:to[i + 1]] for i in range(len(to) - 1)]
        else:
            items = [text[to[i]:to[i + 1]].decode("utf-8") for i in range(len(to) - 1)]
        out = []
        tab = {}
        for i, (ti, size, line, hoff, d, key) in enumerate(zip(
                r["text_idx"].tolist(), r["pcr_size"].tolist(), r["line"].tolist(), r["hash_off"].tolist(),
                r["direct"].tolist(), r["key"].tolist())):
            rec = STSRecord(items[2 * ti], p1s[p1o[i]:p1o[i + 1]], p2s[p2o[i]:p2o[i + 1]], size,
                            items[2 * ti + 1], line, hoff, "+" if d == 43 else "-")
            out.append(rec)
            b = tab.get(key)
            if b is None:
                tab[key] = [rec]
            else:
                b.append(rec)
        list.extend(recs, out)
        dict.update(table, tab)
        recs._src = None
        table._src = None

    def record_texts(self):
        """UTF-8 "id\\talias\\t(direct)" of every record, concatenated, and offsets: the
        formatter's record column (engine.py:437-443), built by the parser
        (mp_sts_record_texts)."""
        return self._blob


class MerPCR:
    """Electronic-PCR STS search (reference: core/engine.py:44)."""

    # sts_records / sts_table: the reference's public containers (engine.py:62-63).  A
    # natively parsed file keeps them lazy (_LazyRecords / _LazyTable) only for the engine's
    # own paths, which read the parser's arrays; a caller that reaches either container gets
    # it fully built, so C-level readers (json, numpy, str.join, PyDict_Next) see every item.
    # From then on the records may be edited in place, and the engine rebuilds its arrays
    # from the record objects (_native_current() is False).
    @property
    def sts_records(self) -> List[STSRecord]:
        recs = self._recs
        if isinstance(recs, _LazyRecords):
            recs._ready()
        return recs

    @sts_records.setter
    def sts_records(self, v):
        self._recs = v

    @property
    def sts_table(self) -> Dict[int, List[STSRecord]]:
        tab = self._table
        if isinstance(tab, _LazyTable):
            tab._ready()
        return tab

    @sts_table.setter
    def sts_table(self, v):
        self._table = v

    def __init__(self, wordsize: int = DEFAULT_WORDSIZE, margin: int = DEFAULT_MARGIN,
                 mismatches: int = DEFAULT_MISMATCHES,
                 three_prime_match: int = DEFAULT_THREE_PRIME_MATCH,
                 iupac_mode: int = DEFAULT_IUPAC_MODE, default_pcr_size: int = DEFAULT_PCR_SIZE,
                 threads: int = DEFAULT_THREADS, max_sts_line_length: int = 1022,
                 device: Optional[int] = None, emulate_chunks: bool = False,
                 devices: Optional[Sequence[int]] = None):
        self.wordsize = wordsize
        self.margin = margin
        self.mismatches = mismatches
        self.three_prime_match = three_prime_match
        self.iupac_mode = iupac_mode
        self.default_pcr_size = default_pcr_size
        self.threads = threads
        self.max_sts_line_length = max_sts_line_length
        # devices: several GPUs of this process share every search (owned-range sharding,
        # RCCL gather; MerPCR(devices=[0, 1, ...]) or the CLI's --gpus N); device is the first
        if devices:
            self.devices = [int(d) for d in devices]
            self.device = self.devices[0]
        else:
            self.device = 0 if device is None else int(device)
            self.devices = [self.device]
        # threads > 1: reproduce the reference's per-chunk output (duplicated overlap
        # hits, chunk-local record ends) instead of the exact T=1 result
        self.emulate_chunks = bool(emulate_chunks)

        self.sts_records: List[STSRecord] = []
        self.sts_table: Dict[int, List[STSRecord]] = {}
        self.max_pcr_size = 0
        self.total_hits = 0
        self._dev_table = None
        self._dev_table_sig = None
        self._codes = CharCodes()
        self.last_search_stats: dict = {}
        # kernel-path selection of the device search (tests; _native.Search.set_options
        # keywords), and the genome/search handles kept across search() calls
        self.search_options: dict = {}
        # layout choices of the device seed table (tests and A/B runs; _native.Table keywords:
        # lds_k, h12, kgrp4, split); empty = the library's own
        self.table_options: dict = {}
        self._dev_genome = None
        self._dev_search = None
        self._dev_search_key = None
        self._dev_genome_dev = None
        self._extra_tables: Dict[int, object] = {}
        self._multi = None
        self._multi_key = None

        self._init_lookup_tables()
        self._validate_parameters()

    # ------------------------------------------------------------------ setup
    def _validate_parameters(self):
        """Parameter bounds and messages of engine.py:80-97."""
        if not (MIN_WORDSIZE <= self.wordsize <= MAX_WORDSIZE):
            raise ValueError(f"Word size must be between {MIN_WORDSIZE} and {MAX_WORDSIZE}")
        if not (MIN_MISMATCHES <= self.mismatches <= MAX_MISMATCHES):
            raise ValueError(f"Number of mismatches must be between {MIN_MISMATCHES} and {MAX_MISMATCHES}")
        if not (MIN_MARGIN <= self.margin <= MAX_MARGIN):
            raise ValueError(f"Margin must be between {MIN_MARGIN} and {MAX_MARGIN}")
        if self.three_prime_match < MIN_THREE_PRIME_MATCH:
            raise ValueError(f"Three prime match must be at least {MIN_THREE_PRIME_MATCH}")
        if not (MIN_PCR_SIZE <= self.default_pcr_size <= MAX_PCR_SIZE):
            raise ValueError(f"Default PCR size must be between {MIN_PCR_SIZE} and {MAX_PCR_SIZE}")

    def _init_lookup_tables(self):
        """Host tables of engine.py:99-191 (scode, compl, iupac_mapping, ambig)."""
        self.scode = [AMBIG] * 256
        for ch, c in _CODE2.items():
            self.scode[ord(ch)] = self.scode[ord(ch.lower())] = c
        self.compl = {}
        for k, v in _COMPL_BASE.items():
            self.compl[k] = v
            self.compl[k.lower()] = v.lower()
        self.iupac_mapping = dict(_IUPAC_SETS)
        self.iupac_mapping.update({k.lower(): v for k, v in _IUPAC_SETS.items()})
        self.ambig = {b: True for b in "BDHKMNRSVWXYbdhkmnrsvwxy"}

    # ------------------------------------------------------------------ STS file
    def load_sts_file(self, filename: str) -> bool:
        """Parse an STS file into oriented records (engine.py:193-302)."""
        start = time.time()
        if os.path.getsize(filename) == 0:
            logger.error(f"STS file '{filename}' is empty")
            return False
        logger.info(f"Reading STS file: {filename}")
        self.sts_records = []
        self.sts_table = {}
        self.max_pcr_size = 0
        self._dev_table = None
        self._native_arrays = None
        if _utf8_locale():
            done = self._load_sts_native(filename, start)
            if done is not None:
                return done
        return self._load_sts_py(filename, start)

    def _load_sts_native(self, filename: str, start: float) -> Optional[bool]:
        """load_sts_file through mp_sts_parse (merpcr_amd/csrc/mp_sts.hip); None when the
        file needs Python's Unicode rules (non-ASCII primer/size fields)."""
        from .. import _native
        r = _native.sts_parse(filename, self.wordsize, self.default_pcr_size)
        if r["status"] == _native.MP_STS_PYTHON:
            return None
        n = r["n"]
        # the record objects are built lazily (_LazyRecords): the search path reads the arrays
        src = _NativeRecords(r)
        src._blob = (r["rec_text"], r["rec_text_off"])
        src.recs = self._recs = _LazyRecords(src, n)
        src.table = self._table = _LazyTable(src)
        self._sts_src = src
        self.max_pcr_size = r["max_pcr_size"]
        self._native_arrays = (self._recs, n, (r["key"], r["hash_off"], r["pcr_size"], r["p1"], r["p1_off"],
                                                     r["p2"], r["p2_off"]))
        if r["status"] == _native.MP_STS_BAD_LINE:
            logger.error(f"Bad STS file format at line {r['bad_line']}. Expected at least 4 fields.")
            return False
        self._log_sts_summary(r["short"], r["ambig"], r["badsize"], start)
        return True

    def _load_sts_py(self, filename: str, start: float) -> bool:
        """load_sts_file restated in Python (engine.py:212-302)."""
        short = ambig = badsize = 0
        W = self.wordsize
        with open(filename, "r") as fh:
            lines = fh.readlines()
        for line_no, raw in enumerate(lines, 1):
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            fields = line.split("\t")
            if len(fields) < 4:
                logger.error(f"Bad STS file format at line {line_no}. Expected at least 4 fields.")
                return False
            sts_id = fields[0]
            p1 = fields[1].upper()
            p2 = fields[2].upper()
            size = self._parse_pcr_size(fields[3])
            alias = fields[4] if len(fields) > 4 else ""
            if len(p1) < W or len(p2) < W:
                short += 1
                continue
            if len(p1) + len(p2) > size:
                badsize += 1
                size = len(p1) + len(p2)
            if size > self.max_pcr_size:
                self.max_pcr_size = size
            off1, key1 = self._hash_value(p1)
            if off1 >= 0:
                self._insert_sts(STSRecord(id=sts_id, primer1=p1, primer2=p2, pcr_size=size,
                                           alias=alias, offset=line_no, hash_offset=off1,
                                           direct="+"), key1)
            else:
                ambig += 1
            rc1 = self._reverse_complement(p1)
            off2, key2 = self._hash_value(p2)
            if off2 >= 0:
                self._insert_sts(STSRecord(id=sts_id, primer1=p2, primer2=rc1, pcr_size=size,
                                           alias=alias, offset=line_no, hash_offset=off2,
                                           direct="-"), key2)
            else:
                ambig += 1
        self._log_sts_summary(short, ambig, badsize, start)
        return True

    def _log_sts_summary(self, short: int, ambig: int, badsize: int, start: float):
        """Warnings and summary of engine.py:289-302."""
        W = self.wordsize
        if short:
            logger.warning(f"{short} STSs have primer shorter than word size ({W}): not included in search")
        if ambig:
            logger.warning(f"{ambig} primers have ambiguities which prevent computation of a hash value: "
                           "not included in search")
        if badsize:
            logger.warning(f"{badsize} STSs have a primer length sum greater than the pcr size: "
                           "expected pcr size adjusted")
        logger.info(f"Loaded {self._n_records()} STS records in {time.time() - start:.2f} seconds")
        return True

    def _parse_pcr_size(self, pcr_size_str: str) -> int:
        """'a-b' -> midpoint, int > 0 as is, else the default (engine.py:304-322)."""
        if "-" in pcr_size_str:
            parts = pcr_size_str.split("-")
            if len(parts) == 2 and parts[0] and parts[1]:
                try:
                    return (int(parts[0]) + int(parts[1])) // 2
                except ValueError:
                    return self.default_pcr_size
            return self.default_pcr_size
        try:
            v = int(pcr_size_str)
        except ValueError:
            return self.default_pcr_size
        return v if v > 0 else self.default_pcr_size

    def _insert_sts(self, sts: STSRecord, hash_value: int):
        """Append to the key's bucket and the flat record list (engine.py:324-329)."""
        self.sts_table.setdefault(hash_value, []).append(sts)
        self.sts_records.append(sts)

    def _hash_value(self, primer: str) -> Tuple[int, int]:
        """(offset, value) of the first all-ACGTU W-mer (engine.py:331-355).

        The reference looks every character it reaches up in its 256-entry scode list, so a
        character whose upper case is beyond U+00FF raises IndexError when the scan reaches
        it: every position up to the end of the first valid window, or, when there is none,
        up to the first ambiguous character at or after len - W (the last offset tried)."""
        p = primer.upper()
        W = self.wordsize
        n = len(p)
        if n < W:
            return -1, 0
        run = 0
        v = 0
        mask = (1 << (2 * W)) - 1
        for i, ch in enumerate(p):
            if ord(ch) > 0xFF:
                raise IndexError("list index out of range")
            c = _CODE2.get(ch)
            if c is None:
                if i >= n - W:
                    return -1, 0
                run = 0
                v = 0
                continue
            v = ((v << 2) | c) & mask
            run += 1
            if run >= W:
                return i - W + 1, v
        return -1, 0

    def _reverse_complement(self, sequence: str) -> str:
        """Reverse complement, unknown characters -> 'N' (engine.py:357-359)."""
        compl = self.compl
        return "".join(compl.get(b, "N") for b in reversed(sequence))

    def _compare_seqs(self, seq1: str, seq2: str, strand: str) -> bool:
        """Host copy of the primer compare rule (engine.py:599-642).

        Kept for API compatibility; the search itself runs this rule on the GPU
        (merpcr_amd/csrc/mp_search.hip, primer_ok)."""
        if len(seq1) != len(seq2):
            return False
        L = len(seq1)
        X = self.three_prime_match
        mm = 0
        for i in range(L):
            a = seq1[i].upper()
            b = seq2[i].upper()
            if self.iupac_mode and a in self.iupac_mapping and b in self.iupac_mapping:
                ok = not set(self.iupac_mapping[a]).isdisjoint(self.iupac_mapping[b])
            else:
                ok = a == b
            if not ok:
                if (strand == "+" and i >= L - X) or (strand == "-" and i < X):
                    return False
                mm += 1
                if mm > self.mismatches:
                    return False
        return True

    def load_fasta_file(self, filename: str, *, on_device: bool = False) -> List[FASTARecord]:
        """FASTA records with the reference's filter (io/fasta.py:18-71).  With on_device=True
        (the CLI, which searches what it reads) a single-device engine ingests large ASCII
        files on its GPU, and the sequences stay there for the search (FASTALoader.load_file's
        device form); by default the records are host strings, as the reference's are."""
        dev = self.device if on_device and len(self.devices) == 1 else None
        return FASTALoader.load_file(filename, device=dev)

    # ------------------------------------------------------------------ device
    def _params(self):
        from .._native import MPParams
        return MPParams(self.wordsize, self.margin, self.mismatches, self.three_prime_match,
                        self.iupac_mode)

    def _n_records(self) -> int:
        """len(sts_records), without building a lazy list's records."""
        recs = self._recs
        n = recs.native_len() if isinstance(recs, _LazyRecords) else None
        return len(recs) if n is None else n

    def _native_current(self) -> bool:
        """sts_records is the native parser's and has never been handed out: no caller can
        have edited it (nor a record in it), so the parser's arrays and texts are current."""
        na = getattr(self, "_native_arrays", None)
        recs = self._recs
        return (na is not None and na[0] is recs and isinstance(recs, _LazyRecords) and recs._src is not None
                and recs.native_len() == na[1])

    def _records_sig(self):
        """What the device table and the formatter's record column depend on: the parser's
        arrays while they are current, else the records' content (edits in place included)."""
        if self._native_current():
            return ("native", id(self._recs))
        return ("objects", hash(tuple((r.id, r.alias, r.direct, r.primer1, r.primer2, r.pcr_size, r.hash_offset)
                                      for r in self._recs)))

    def _record_keys(self, recs) -> np.ndarray:
        """Each record's seed key: the one it is filed under in sts_table.  The reference finds a
        record only through its load-time bucket (engine.py:265-279, 483-486), whatever its
        primer holds after an edit in place, and takes hash_offset from the record itself.

        Deliberate extension, not reference parity: the device table is built from sts_records,
        so a record the caller put in sts_records alone (never filed in sts_table) is keyed by
        its primer as the loader would have keyed it and IS searched, where the reference, which
        walks only sts_table's buckets (engine.py:483-486), would never report it; conversely a
        record filed in sts_table alone is not searched here.  Both need the caller to edit the
        engine's internal containers by hand; the loaders keep the two in step."""
        filed = {}
        for h, lst in self.sts_table.items():
            for r in lst:
                filed.setdefault(id(r), h)
        return np.fromiter((filed[id(r)] if id(r) in filed else self._hash_value(r.primer1)[1] for r in recs),
                           dtype=np.uint32, count=len(recs))

    def _table_arrays(self):
        """Record arrays for mp_table_create in sts_records order."""
        recs = self._recs
        na = getattr(self, "_native_arrays", None)
        if self._native_current():
            return na[2]
        key = self._record_keys(recs)
        hash_off = np.fromiter((r.hash_offset for r in recs), dtype=np.uint32, count=len(recs))
        size = np.fromiter((r.pcr_size for r in recs), dtype=np.uint64, count=len(recs))
        p1 = [self._codes.primer_bytes(r.primer1) for r in recs]
        p2 = [self._codes.primer_bytes(r.primer2) for r in recs]
        p1_off = np.zeros(len(recs) + 1, dtype=np.uint64)
        p2_off = np.zeros(len(recs) + 1, dtype=np.uint64)
        if recs:
            np.cumsum([len(b) for b in p1], out=p1_off[1:])
            np.cumsum([len(b) for b in p2], out=p2_off[1:])
        return (key, hash_off, size, np.frombuffer(b"".join(p1), dtype=np.uint8), p1_off,
                np.frombuffer(b"".join(p2), dtype=np.uint8), p2_off)

    def device_table(self):
        """The seed table resident on this engine's GPU (rebuilt when stale)."""
        from .. import _native
        sig = (self._records_sig(), self._n_records(), self.wordsize, self.margin,
               self.mismatches, self.three_prime_match, self.iupac_mode, self.device,
               tuple(sorted(self.table_options.items())))
        if self._dev_table is None or self._dev_table_sig != sig:
            self._dev_table = _native.Table(self._params(), self.device, *self._table_arrays(), **self.table_options)
            self._dev_table_sig = sig
            self._extra_tables = {}
        return self._dev_table

    def prepare_device(self):
        """Build the seed table(s) on the device now -- the HIP runtime starts with them --
        so that search() finds them ready.  The CLI runs this on a thread beside the FASTA
        read (both are native calls that release the GIL).  A failure is left for search() to
        raise at its own point of the run, as without the head start."""
        try:
            if len(self.devices) > 1:
                self.device_tables()
            else:
                self.device_table()
        except Exception:  # noqa: BLE001 -- search() repeats the call and raises it there
            pass

    def device_tables(self) -> list:
        """One seed table per entry of self.devices (a repeated device shares its table)."""
        from .. import _native
        first = self.device_table()
        out = []
        for d in self.devices:
            if d == self.device:
                out.append(first)
                continue
            if d not in self._extra_tables:
                self._extra_tables[d] = _native.Table(self._params(), d, *self._table_arrays(), **self.table_options)
            out.append(self._extra_tables[d])
        return out

    def encode_sequences(self, sequences: Sequence[str]) -> List[np.ndarray]:
        """Device bytes of each sequence, in the coordinates of ``seq.upper()``.

        Raises IndexError as the reference's scan does (engine.py:455-503 looks every base
        up in the 256-entry scode list): a sequence longer than W holding a character whose
        upper case is beyond U+00FF."""
        out = []
        W = self.wordsize
        for s in sequences:
            if not s.isascii():
                up = s.upper()
                if len(up) > W and max(map(ord, up)) > 0xFF:
                    raise IndexError("list index out of range")
            out.append(self._codes.sequence_bytes(s))
        return out

    def encode_records(self, fasta_records: Sequence[FASTARecord]) -> List[np.ndarray]:
        """encode_sequences of the records' sequences; a record from the native FASTA
        reader hands over its ASCII bytes as they are (no str round trip)."""
        out = []
        for r in fasta_records:
            span = _device_span(r)
            if span is not None and span.device == self.device and len(self.devices) == 1:
                out.append(span)  # packed where it is (mp_genome_put_device)
                continue
            raw = _raw_ascii(r)
            out.append(np.frombuffer(raw, dtype=np.uint8) if raw is not None else
                       self.encode_sequences([r.sequence])[0])
        return out

    def chunk_plan(self, seq_len: int) -> List[Tuple[int, int]]:
        """(offset, length) of each chunk the reference's search scans for a record of
        seq_len bases (engine.py:380-410): T = threads for records of >= 100 kbp, reduced
        while (T+1)*overlap > n; each chunk overlaps the next by max_pcr_size + M - 1."""
        t = self.threads if seq_len >= MIN_FILESIZE_FOR_THREADING else 1
        overlap = self.max_pcr_size + self.margin - 1
        while t > 1 and (t + 1) * overlap > seq_len:
            t -= 1
        size = int((seq_len - (t + 1) * overlap) / t) + 2 * overlap
        plan, off = [], 0
        for i in range(t):
            ln = size if i < t - 1 else seq_len - off
            plan.append((off, ln))
            off += ln - overlap
        return plan

    def find_hits(self, fasta_records: Sequence[FASTARecord]) -> np.ndarray:
        """All hits of all records on the GPU, in output order.

        Returns the structured array of mp_hit (pos1, pos2, seq, rec).  With
        emulate_chunks and threads > 1, every chunk of the reference's plan is searched
        as its own sequence, hits are shifted to record coordinates, and each record's
        chunk lists are concatenated in chunk order and stably sorted on pos1
        (engine.py:412-434) -- overlap hits then appear once per chunk, as in the
        reference's multi-process output."""
        self.device_table()  # registers the primers' non-ASCII codes before the genome is encoded
        return self._hits_of(self.encode_records(fasta_records))

    def _hits_of(self, data: List[np.ndarray]) -> np.ndarray:
        if not (self.emulate_chunks and self.threads > 1):
            return self._search_device(data)
        pieces, owner, base = [], [], []
        for i, d in enumerate(data):
            for off, ln in self.chunk_plan(len(d)):
                pieces.append(d[off:off + ln])
                owner.append(i)
                base.append(off)
        hits = self._search_device(pieces)
        if len(hits):
            piece = hits["seq"].astype(np.int64)
            shift = np.asarray(base, dtype=np.uint64)[piece]
            hits["pos1"] += shift
            hits["pos2"] += shift
            hits["seq"] = np.asarray(owner, dtype=np.uint32)[piece]
            # LSD: stable on pos1, then stable on the record -> chunk order kept on ties
            hits = hits[np.argsort(hits["pos1"], kind="stable")]
            hits = hits[np.argsort(hits["seq"], kind="stable")]
        return hits

    def _device_search(self, lengths):
        """Genome and search handles of this engine, kept across calls: the genome is
        re-laid out on its existing device buffers (mp_genome_reset) and the search keeps
        its grown hit lists and sort buffers."""
        from .. import _native
        table = self.device_table()
        if self._dev_genome is None or self._dev_genome_dev != self.device:
            self._dev_search = None
            self._dev_genome = _native.Genome(self.device, lengths)
            self._dev_genome_dev = self.device
        else:
            self._dev_genome.reset(lengths)
        key = tuple(sorted(self.search_options.items()))
        if self._dev_search is None or self._dev_search.table is not table or self._dev_search_key != key:
            if self._dev_search is not None:
                self._dev_search.close()
            self._dev_search = _native.Search(table, self._dev_genome)
            if self.search_options:
                self._dev_search.set_options(**self.search_options)
            self._dev_search_key = key
        return self._dev_genome, self._dev_search

    def _search_multi(self, data: Sequence[np.ndarray]) -> np.ndarray:
        """Several devices: owned (sequence, k) ranges of equal base count, one per device,
        searched in parallel and gathered into devices[0] (mp_multi_*, RCCL)."""
        from .. import _native
        tables = self.device_tables()
        key = (tuple(self.devices), tuple(id(tb) for tb in tables), tuple(sorted(self.search_options.items())))
        if self._multi is None or self._multi_key != key:
            if self._multi is not None:
                self._multi.close()
            self._multi = _native.Multi(self.devices, tables)
            self._multi_key = key
            self._multi_opts_pending = bool(self.search_options)
        m = self._multi
        m.genome([len(d) for d in data])
        if self._multi_opts_pending:  # the per-device searches exist once the genome is laid out
            for i in range(len(self.devices)):
                m.device(i)[0].set_options(**self.search_options)
            self._multi_opts_pending = False
        for i, d in enumerate(data):
            if len(d):
                m.put(i, d)
        m.seal()
        t0 = time.time()
        n = m.run()
        hits = m.fetch(n)
        per = []
        for i in range(len(self.devices)):
            s, rng, gms = m.device(i)
            per.append(dict(s.last_stats(), owned=rng))
        self.last_search_stats = dict(wall_s=time.time() - t0, hits=n, gather_ms=gms, devices=per,
                                      scan_ms=max(p["scan_ms"] for p in per), regrowths=0)
        return hits

    def _search_device(self, data: Sequence[np.ndarray]) -> np.ndarray:
        if len(self.devices) > 1:
            return self._search_multi(data)
        genome, search = self._device_search([len(d) for d in data])
        from .._native import DeviceSpan
        for i, d in enumerate(data):
            if len(d):
                if isinstance(d, DeviceSpan):
                    genome.put_device(i, d.ptr, len(d))
                else:
                    genome.put(i, d)
        genome.seal()
        t0 = time.time()
        n = search.run()
        hits = search.fetch(n)
        self.last_search_stats = dict(search.last_stats(), wall_s=time.time() - t0, hits=n,
                                      regrowths=search.regrowths())
        return hits

    # ------------------------------------------------------------------ search
    def _log_thread_plan(self, seq_len: int):
        """Reference's per-record thread-planning log lines (engine.py:380-392)."""
        t = self.threads
        if seq_len < MIN_FILESIZE_FOR_THREADING:
            logger.info("Sequence too small for threading, using single thread.")
            t = 1
        overlap = self.max_pcr_size + self.margin - 1
        while t > 1 and (t + 1) * overlap > seq_len:
            t -= 1
            logger.info(f"Reduced threads to {t} due to sequence size limitations")

    def format_bytes(self, fasta_records: Sequence[FASTARecord], hits: np.ndarray) -> bytes:
        """The output text of engine.py:437-443 for `hits`, UTF-8, by mp_format_hits."""
        from .. import _native
        return _native.Formatter([r.label for r in fasta_records], *self._record_texts())(hits)

    def _record_texts(self):
        """The formatter's record column (UTF-8 "id\talias\t(direct)" per record, and
        offsets): from the parser's bytes while the records are the native parser's and
        unseen by callers, else from the record objects."""
        if self._native_current():
            return self._sts_src.record_texts()
        from .._native import _csr
        # rebuilt on every call from the current record objects, as engine.py:437-443 reads them
        return _csr([f"{r.id}\t{r.alias}\t({r.direct})" for r in self._recs])

    def format_hits(self, fasta_records: Sequence[FASTARecord], hits: np.ndarray) -> List[str]:
        """Output lines exactly as engine.py:437-443 prints them."""
        text = self.format_bytes(fasta_records, hits).decode("utf-8")
        return text.split("\n")[:-1] if text else []

    def hits_as_objects(self, hits: np.ndarray) -> List[STSHit]:
        recs = self.sts_records
        return [STSHit(pos1=int(h["pos1"]), pos2=int(h["pos2"]), sts=recs[int(h["rec"])]) for h in hits]

    def search(self, fasta_records: List[FASTARecord], output_file: str = None) -> int:
        """Search every record; print one line per hit (engine.py:365-451).

        One device pass covers all records; the per-record log lines and output then follow
        in the reference's order (record i's lines before record i+1's log).  A record the
        reference's scan would fail on (IndexError, see encode_sequences) ends the call
        after the output of the records before it, as in the reference."""
        to_file = bool(output_file) and output_file.lower() != "stdout"
        output = open(output_file, "w") if to_file else sys.stdout
        total = 0
        try:
            recs = list(fasta_records)
            self.device_table()
            data, err = [], None
            for r in recs:
                try:
                    data.extend(self.encode_records([r]))
                except IndexError as e:
                    err = e
                    break
            n_ok = len(data)
            if self.threads > 1 and not self.emulate_chunks and any(
                    len(self.chunk_plan(_seq_len(r))) > 1 for r in recs[:n_ok]):
                logger.warning("threads > 1: hits are reported once, as with -T 1 (the reference's "
                               "multi-process chunking repeats hits inside chunk overlaps; "
                               "emulate_chunks=True reproduces that output)")
            hits = self._hits_of(data) if n_ok else np.zeros(0, dtype=_hit_dtype())
            text = self.format_bytes(recs[:n_ok], hits) if len(hits) else b""
            # byte range of each record's lines: hits are ordered by record
            per = np.bincount(hits["seq"].astype(np.int64), minlength=n_ok) if len(hits) else np.zeros(n_ok, np.int64)
            ends = np.flatnonzero(np.frombuffer(text, dtype=np.uint8) == 10) + 1 if text else np.zeros(0, np.int64)
            line_end = np.cumsum(per)
            pos = 0
            for i, rec in enumerate(recs[:n_ok]):
                logger.info(f"Processing sequence: {rec.label} ({_seq_len(rec)} bp)")
                self._log_thread_plan(_seq_len(rec))
                if per[i]:
                    stop = int(ends[line_end[i] - 1])
                    output.write(text[pos:stop].decode("utf-8"))
                    pos = stop
                    total += int(per[i])
            if err is not None:
                rec = recs[n_ok]
                logger.info(f"Processing sequence: {rec.label} ({_seq_len(rec)} bp)")
                self._log_thread_plan(_seq_len(rec))
                raise err
        finally:
            if to_file:
                output.close()
        logger.info(f"Total hits found: {total}")
        self.total_hits = total
        return total

    # kept for surface compatibility with code that drives one chunk by hand
    def _process_thread(self, thread_data: ThreadData) -> ThreadData:
        """One chunk scanned as its own sequence (engine.py:453-505), on the GPU: always one
        device sequence, whatever threads / emulate_chunks say."""
        self.device_table()
        hits = self._search_device(self.encode_sequences([thread_data.sequence]))
        for h in self.hits_as_objects(hits):
            h.pos1 += thread_data.offset
            h.pos2 += thread_data.offset
            thread_data.hits.append(h)
        return thread_data


def _raw_ascii(rec):
    f = getattr(rec, "raw_ascii", None)
    return f() if f is not None else None


def _device_span(rec):
    f = getattr(rec, "device_span", None)
    return f() if f is not None else None


def _seq_len(rec) -> int:
    span = _device_span(rec)
    if span is not None:
        return len(span)
    raw = _raw_ascii(rec)
    return len(raw) if raw is not None else len(rec.sequence)


def _hit_dtype():
    from .._native import HIT_DTYPE
    return HIT_DTYPE
