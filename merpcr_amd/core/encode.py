"""Byte encoding of primers and sequences for the device.

The device compares bytes.  ASCII characters pass through (the device
upper-cases a-z, matching ``str.upper()`` at engine.py:455 and the per-character
``.upper()`` of engine.py:616-631).  Non-ASCII characters -- possible only for
sequences handed to ``search`` directly, or the FASTA filter's U+017F -- are
first upper-cased in Python exactly as the reference does, then mapped to opaque
bytes: every distinct non-ASCII primer character gets its own code in
0x80..0xFE, and any other non-ASCII genome character becomes 0xFF, which no
primer byte equals.  Opaque bytes are not IUPAC symbols, so they only ever match
an identical character -- the reference's literal-equality rule for them.
"""

from __future__ import annotations

from typing import Dict

import numpy as np

UNMATCHED = 0xFF


class CharCodes:
    def __init__(self):
        self.codes: Dict[str, int] = {}

    def _code(self, ch: str, register: bool) -> int:
        c = self.codes.get(ch)
        if c is None:
            if not register:
                return UNMATCHED
            if len(self.codes) >= 0x7F:
                raise ValueError("more than 127 distinct non-ASCII primer characters")
            c = 0x80 + len(self.codes)
            self.codes[ch] = c
        return c

    def primer_bytes(self, primer: str) -> bytes:
        """Primer (already upper-cased by the loader) -> device bytes."""
        if primer.isascii():
            return primer.encode("ascii")
        return bytes(ord(ch) if ord(ch) < 0x80 else self._code(ch, True) for ch in primer)

    def sequence_bytes(self, seq: str) -> np.ndarray:
        """Sequence -> uint8 array in the coordinates of ``seq.upper()``."""
        if seq.isascii():
            return np.frombuffer(seq.encode("ascii"), dtype=np.uint8)
        up = seq.upper()
        return np.fromiter((ord(ch) if ord(ch) < 0x80 else self._code(ch, False) for ch in up),
                           dtype=np.uint8, count=len(up))
