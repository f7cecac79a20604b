"""merpcr_amd -- MI355X-native electronic-PCR STS search.

Drop-in for the merpcr package surface (``MerPCR``, ``STSRecord``,
``FASTARecord``, ``STSHit``; src/merpcr/__init__.py:11-14 of the reference)
whose search hot path runs as HIP kernels on AMD Instinct MI355X (gfx950).
"""

__version__ = "1.0.0"

from .core.engine import MerPCR
from .core.models import FASTARecord, STSHit, STSRecord

__all__ = ["MerPCR", "STSRecord", "FASTARecord", "STSHit"]
