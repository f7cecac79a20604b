"""Core engine and models."""

from .engine import MerPCR
from .models import FASTARecord, STSHit, STSRecord, ThreadData

__all__ = ["MerPCR", "STSRecord", "FASTARecord", "STSHit", "ThreadData"]
