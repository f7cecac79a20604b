"""Data models crossing the search boundary.

Same fields and behaviour as the reference's dataclasses
(src/merpcr/core/models.py:10-69) so user code and tests written against merpcr
see identical objects.
"""

from dataclasses import dataclass, field
from enum import Enum
from typing import List


class SeqType(Enum):
    """Sequence type (models.py:10-14; unused by the search path)."""

    AMINO_ACID = 1
    NUCLEOTIDE = 2


@dataclass
class STSRecord:
    """One oriented STS record (models.py:17-29)."""

    id: str
    primer1: str
    primer2: str
    pcr_size: int
    alias: str = ""
    offset: int = 0
    hash_offset: int = 0
    direct: str = "+"
    ambig_primer: int = 0


@dataclass
class FASTARecord:
    """A FASTA sequence; label = first word of the defline (models.py:32-49)."""

    defline: str
    sequence: str
    label: str = ""

    def __post_init__(self):
        if not self.label:
            d = self.defline.strip()
            if ">" in self.defline:
                d = d[1:]
            self.label = d.split()[0]


@dataclass
class STSHit:
    """A hit: 0-based amplicon start/end and the record (models.py:52-58)."""

    pos1: int
    pos2: int
    sts: STSRecord


@dataclass
class ThreadData:
    """Per-chunk work unit of the reference's scan (models.py:61-69)."""

    thread_id: int
    sequence: str
    offset: int
    length: int
    hits: List[STSHit] = field(default_factory=list)
