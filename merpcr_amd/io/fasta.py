"""FASTA loading with the reference's exact character filter.

The filter defines the coordinate system of every hit: io/fasta.py:60 of the
reference keeps a character c iff ``c.upper() in "ACGTBDHKMNRSVWXY"``.  Over all
of Unicode that is the 32 ASCII letters below plus U+017F (long s, upper 'S');
U is dropped.  Lines are stripped, blank lines skipped, '>' starts a record,
sequence lines before the first header are discarded (fasta.py:42-66).

``FASTALoader.load_file`` reads through the native reader of libmerpcr_hip.so
(``mp_fasta_load``, merpcr_amd/csrc/mp_fasta.hip), which restates that loop in C++
for UTF-8 text (the locale encoding of the reference's ``open(filename, "r")``).
``load_file_py`` is the same loop in Python; it serves non-UTF-8 locales and the
parity tests.
"""

import codecs
import locale
import logging
import os
import re
import time
from typing import List

from ..core.models import FASTARecord

logger = logging.getLogger("merpcr.io.fasta")  # the reference module's logger name

KEEP_CHARS = "ABCDGHKMNRSTVWXYabcdghkmnrstvwxyſ"
_DROP = re.compile("[^" + re.escape(KEEP_CHARS) + "]+")


def _utf8_locale() -> bool:
    """True when open(filename, "r") decodes UTF-8, as the native reader does."""
    return codecs.lookup(locale.getpreferredencoding(False)).name == "utf-8"


def filter_line(line: str) -> str:
    """Keep only the characters the reference's FASTA filter keeps."""
    if line.isascii() and not _DROP.search(line):
        return line
    return _DROP.sub("", line)


class ReaderRecord(FASTARecord):
    """A FASTARecord from the native reader: the sequence stays the reader's filtered UTF-8
    bytes, and the str the reference's API exposes is built on first access.  The device
    path (MerPCR.search / find_hits) encodes ASCII bytes directly, so the CLI never pays
    the bytes -> str -> bytes round trip (about 1.4 s per Gbp)."""

    def __init__(self, defline: str, raw, ascii=None):
        self._raw = raw  # bytes, or a memoryview of the reader's own buffer
        self._ascii = ascii
        self._str = None
        super().__init__(defline=defline, sequence=None)

    @property
    def sequence(self) -> str:
        if self._str is None:
            self._str = str(self._raw, "utf-8")
        return self._str

    @sequence.setter
    def sequence(self, value):
        if value is not None:  # assigned by the caller: the bytes no longer describe it
            self._str = value
            self._raw = None

    def __eq__(self, other):  # equal to a plain FASTARecord with the same fields
        if isinstance(other, FASTARecord):
            return (self.defline, self.sequence, self.label) == (other.defline, other.sequence, other.label)
        return NotImplemented

    __hash__ = None

    def __reduce__(self):
        # pickle / copy / deepcopy as the reference's plain dataclass: _raw may be a view of
        # the native reader's buffer, which neither pickles nor outlives the reader
        return (FASTARecord, (self.defline, self.sequence, self.label))

    def __repr__(self):
        return f"FASTARecord(defline={self.defline!r}, sequence={self.sequence!r}, label={self.label!r})"

    def raw_ascii(self):
        """The sequence as ASCII bytes (or a view of them) without building the str, or None."""
        if self._str is None and self._raw is not None:
            if self._ascii is None:  # the only non-ASCII bytes the filter keeps are U+017F's
                self._ascii = bytes(self._raw).isascii()
            if self._ascii:
                return self._raw
        return None


class DeviceRecord(ReaderRecord):
    """A FASTARecord whose filtered sequence lives in device memory (mp_fasta_load_device):
    the search packs it there (mp_genome_put_device), and the str or bytes of the
    reference's API are copied to the host only when asked for."""

    def __init__(self, defline: str, span):
        self._span = span
        super().__init__(defline, None, True)

    def device_span(self):
        """The sequence's DeviceSpan while it is unmodified, else None."""
        return self._span if self._str is None else None

    def raw_ascii(self):
        if self._str is None and self._raw is None and self._span is not None:
            self._raw = self._span.host()
        return super().raw_ascii()

    @property
    def sequence(self) -> str:
        if self._str is None:
            self.raw_ascii()
        return ReaderRecord.sequence.fget(self)

    @sequence.setter
    def sequence(self, value):
        if value is not None:
            self._span = None
        ReaderRecord.sequence.fset(self, value)


# Files of at least this many bytes are ingested on the device when the caller names one
# (MerPCR's single-device search); smaller ones are read on the host.
DEVICE_MIN_BYTES = int(os.environ.get("MERPCR_DEVICE_FASTA_MIN", str(16 << 20)))


class FASTALoader:
    """Loads FASTA files into FASTARecord lists (reference: io/fasta.py:15-71)."""

    @staticmethod
    def load_file(filename: str, _chunk_bytes: int = 0, device=None) -> List[FASTARecord]:
        """`device`: ingest an ASCII file of DEVICE_MIN_BYTES or more on that GPU
        (mp_fasta_load_device, the same records; the sequences stay in device memory)."""
        if not _utf8_locale():
            return FASTALoader.load_file_py(filename)
        from .. import _native
        start = time.time()
        size = os.path.getsize(filename)
        if size == 0:
            logger.error(f"FASTA file '{filename}' is empty")
            return []
        logger.info(f"Reading FASTA file: {filename}")
        records = None
        if device is not None and not _chunk_bytes and size >= DEVICE_MIN_BYTES:
            try:
                got = _native.fasta_read_device(filename, int(device))
            except _native.NativeError as e:  # no usable device: the host reader
                logger.debug(f"device FASTA ingestion unavailable ({e}); reading on the host")
                got = None
            if got is not None:
                records = [DeviceRecord(defline, span) for defline, span in got]
        if records is None:
            records = []
            for defline, seq, ascii in _native.fasta_read(filename, _chunk_bytes, with_ascii=True):
                records.append(ReaderRecord(defline, seq, ascii))
        logger.info(f"Loaded {len(records)} sequences in {time.time() - start:.2f} seconds")
        return records

    @staticmethod
    def load_file_py(filename: str) -> List[FASTARecord]:
        start = time.time()
        if os.path.getsize(filename) == 0:
            logger.error(f"FASTA file '{filename}' is empty")
            return []
        logger.info(f"Reading FASTA file: {filename}")
        records: List[FASTARecord] = []
        head = None
        parts: List[str] = []
        with open(filename, "r") as fh:
            for raw in fh:
                line = raw.strip()
                if not line:
                    continue
                if line[0] == ">":
                    if head is not None:
                        records.append(FASTARecord(defline=head, sequence="".join(parts)))
                    head = line
                    parts = []
                elif head is not None:
                    parts.append(filter_line(line))
        if head is not None:
            records.append(FASTARecord(defline=head, sequence="".join(parts)))
        logger.info(f"Loaded {len(records)} sequences in {time.time() - start:.2f} seconds")
        return records
