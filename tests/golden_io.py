"""Helpers that read the committed golden fixtures (data only)."""

import functools
import gzip
import json
import os

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@functools.lru_cache(maxsize=None)
def load_golden(name):
    with gzip.open(os.path.join(GOLDEN_DIR, name), "rt") as fh:
        return json.load(fh)


def data_path(name):
    return os.path.join(GOLDEN_DIR, "data", name)


def case_inputs(case):
    """(params, sts_lines, [(label, seq)]) for one golden case, FASTA filtered by the oracle."""
    from oracle import epcr_oracle as O
    sts_lines = case["sts_text"].splitlines(keepends=True)
    if "fasta_text" in case:
        import io
        recs = O.fasta_from_lines(io.StringIO(case["fasta_text"], newline=None))
        recs = [(O.fasta_label(d), s) for d, s in recs]
    else:
        recs = [(O.fasta_label(d), s) for d, s in case["records"]]
    return case["params"], sts_lines, recs
