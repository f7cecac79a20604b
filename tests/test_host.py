"""Host-side surface of the drop-in (no GPU): loaders, helpers, CLI, parameter bounds.

Expected values come from the reference's golden outputs (tests/golden) and
from its own unit tests (tests/test_engine_internals.py,
tests/test_io_modules.py, tests/test_cli_enhanced.py of the reference).
"""

import io
import os
import tempfile

import pytest

from merpcr_amd import FASTARecord, MerPCR, STSHit, STSRecord
from merpcr_amd.cli import convert_mepcr_arguments, create_parser
from merpcr_amd.io.fasta import FASTALoader
from tests.golden_io import data_path, load_golden


def test_unit_kats_through_engine_helpers():
    k = load_golden("unit_kats.json.gz")
    for p, W, exp in k["hash"]:
        assert list(MerPCR(wordsize=W)._hash_value(p)) == exp
    e = MerPCR()
    for s, exp in k["revcomp"]:
        assert e._reverse_complement(s) == exp
    for a, b, strand, N, X, I, exp in k["compare"]:
        assert MerPCR(mismatches=N, three_prime_match=X, iupac_mode=I)._compare_seqs(a, b, strand) == exp
    for f, exp in k["pcr_size"]:
        assert MerPCR(default_pcr_size=240)._parse_pcr_size(f) == exp


def test_sts_loader_matches_reference_counts():
    for case in load_golden("random_cases.json.gz")["cases"]:
        e = MerPCR(**case["params"])
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "x.sts")
            with open(p, "w") as fh:
                fh.write(case["sts_text"])
            ok = e.load_sts_file(p)
        assert ok == case["load_ok"]
        if ok:
            assert e.max_pcr_size == case["max_pcr_size"]
            assert len(e.sts_records) == case["n_records"]
            assert sum(len(v) for v in e.sts_table.values()) == len(e.sts_records)


def test_fasta_loader_matches_reference():
    for case in load_golden("random_cases.json.gz")["cases"]:
        if "fasta_text" not in case or not case["load_ok"]:
            continue
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "x.fa")
            with open(p, "w", newline="") as fh:
                fh.write(case["fasta_text"])
            recs = FASTALoader.load_file(p)
        assert [[r.defline, r.sequence, r.label] for r in recs] == case["fasta"]


def test_fasta_filter_kat_and_bundled():
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "f.fa")
        with open(p, "w") as fh:
            fh.write(">filtered\nATCG123NNNN456ATCG\nWXYZ789GCTA\n")
        assert FASTALoader.load_file(p)[0].sequence == "ATCGNNNNATCGWXYGCTA"
        open(os.path.join(td, "e.fa"), "w").close()
        assert FASTALoader.load_file(os.path.join(td, "e.fa")) == []
    recs = MerPCR().load_fasta_file(data_path("test.fa"))
    assert len(recs) == 1 and recs[0].label == "L78833" and len(recs[0].sequence) == 117143


def test_parameter_bounds():
    MerPCR(wordsize=3, margin=0, mismatches=0, three_prime_match=0)
    MerPCR(wordsize=16, margin=10000, mismatches=10)
    for kw in (dict(wordsize=2), dict(wordsize=17), dict(mismatches=-1), dict(mismatches=11),
               dict(margin=-1), dict(margin=20000), dict(default_pcr_size=0),
               dict(default_pcr_size=15000), dict(three_prime_match=-1)):
        with pytest.raises(ValueError):
            MerPCR(**kw)


def test_models():
    r = FASTARecord(defline=">seq1 some description", sequence="ACGT")
    assert r.label == "seq1"
    assert FASTARecord(defline="noangle x", sequence="").label == "noangle"
    s = STSRecord(id="a", primer1="AC", primer2="GT", pcr_size=10)
    assert s.direct == "+" and s.hash_offset == 0
    assert STSHit(pos1=1, pos2=2, sts=s).sts is s


def test_cli_conversion_and_defaults():
    assert convert_mepcr_arguments(["M=50", "N=1", "W=8", "P=1", "-help", "x.sts"]) == \
        ["-M", "50", "-N", "1", "-W", "8", "--help", "x.sts"]
    a = create_parser().parse_args(["a.sts", "b.fa"])
    assert (a.margin, a.mismatches, a.wordsize, a.threads, a.three_prime_match, a.quiet,
            a.default_pcr_size, a.iupac, a.max_sts_line_length) == (50, 0, 11, 1, 1, 1, 240, 0, 1022)
    for bad in (["-M", "10001"], ["-N", "11"], ["-W", "2"], ["-T", "0"], ["-Z", "0"]):
        with pytest.raises(SystemExit):
            create_parser().parse_args(["a.sts", "b.fa"] + bad)


def test_cli_fails_cleanly_on_bad_sts(capsys):
    from merpcr_amd.cli import main
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "bad.sts")
        with open(p, "w") as fh:
            fh.write("ONLY\tTHREE\tFIELDS\n")
        assert main([p, data_path("test.fa")]) == 1


def test_chunk_plan_matches_oracle():
    """MerPCR.chunk_plan restates engine.py:380-410 like oracle.chunk_plan does."""
    import random as _r
    from oracle import epcr_oracle as O
    g = _r.Random(5)
    for _ in range(2000):
        n = g.choice([0, 1, 99999, 100000, 100001, g.randint(0, 10**7), g.randint(10**5, 10**6)])
        t = g.randint(1, 64)
        eng = MerPCR(threads=t, margin=g.randint(0, 10000))
        eng.max_pcr_size = g.randint(6, 20000)
        plan = eng.chunk_plan(n)
        assert plan == O.chunk_plan(n, t, eng.max_pcr_size, eng.margin)
        assert plan[0][0] == 0 and plan[-1][0] + plan[-1][1] == n
