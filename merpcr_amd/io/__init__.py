"""Input loaders."""

from .fasta import FASTALoader

__all__ = ["FASTALoader"]
