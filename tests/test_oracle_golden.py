"""Pin the CPU oracle (oracle/epcr_oracle.py) against the reference's outputs.

Fixtures in tests/golden/ were produced by running the reference itself
(tests/golden/make_golden.py).  Unit KATs restate values from the reference's
own tests (tests/test_engine_internals.py:26-154,
tests/test_utils_comprehensive.py:173-181, tests/test_io_modules.py:88-100).
"""

import io

import pytest

from oracle import epcr_oracle as O
from tests.golden_io import case_inputs, data_path, load_golden


def _run(case, threads=1):
    params, sts_lines, recs = case_inputs(case)
    table = O.load_sts_lines(sts_lines, params["wordsize"], params["default_pcr_size"])
    if table is None:
        return None, None
    p = O.params(**params)
    return table, O.search_lines(recs, table, p, threads=threads)


def _expected_lines(case):
    return case["output"].splitlines()


def test_reference_unit_kats():
    # test_engine_internals.py:26-67 and test_utils_comprehensive.py:173-181
    assert O.hash_word("AAAAAAAA", 8) == (0, 0)
    assert O.hash_word("TTTTTTTT", 8) == (0, 65535)
    assert O.hash_word("ATCGATNG", 8)[0] == -1
    assert O.hash_word("NNNATCGATCGATCG", 8)[0] == 3
    assert O.hash_word("ATCG", 8)[0] == -1
    assert O.hash_word("ATCG", 4) == (0, 54)
    # test_engine_internals.py:165-195
    assert O.revcomp("ATCGN") == "NCGAT"
    assert O.revcomp("RWYS") == "SRWY"
    assert O.revcomp("AtCg") == "cGaT"
    # test_engine_internals.py:78-154
    assert O.primer_match("ATCGATCG", "TTCGATCG", "+", 1, 2, 0)
    assert not O.primer_match("ATCGATCG", "ATCGATCT", "+", 1, 2, 0)
    assert not O.primer_match("ATCGATCG", "AGCGATCG", "-", 1, 2, 0)
    assert O.primer_match("ATCG", "RTCG", "+", 0, 1, 1)
    assert not O.primer_match("CTCG", "RTCG", "+", 0, 1, 1)
    assert not O.primer_match("ACCG", "AWCG", "+", 0, 1, 1)


def test_generated_unit_kats():
    k = load_golden("unit_kats.json.gz")
    for p, W, exp in k["hash"]:
        assert list(O.hash_word(p, W)) == exp, (p, W)
    for s, exp in k["revcomp"]:
        assert O.revcomp(s) == exp, s
    for a, b, strand, N, X, I, exp in k["compare"]:
        assert O.primer_match(a, b, strand, N, X, I) == exp, (a, b, strand, N, X, I)
    for f, exp in k["pcr_size"]:
        assert O.parse_pcr_size(f, 240) == exp, f


def test_fasta_filter_kat():
    # test_io_modules.py:88-100
    recs = O.fasta_from_lines(io.StringIO(">filtered\nATCG123NNNN456ATCG\nWXYZ789GCTA\n"))
    assert recs == [(">filtered", "ATCGNNNNATCGWXYGCTA")]


def test_bundled_data():
    g = load_golden("bundled.json.gz")
    import hashlib
    sts = open(data_path("test.sts")).read()
    fa = open(data_path("test.fa")).read()
    assert hashlib.sha256(sts.encode()).hexdigest() == g["sts_sha256"]
    assert hashlib.sha256(fa.encode()).hexdigest() == g["fa_sha256"]
    recs = [(O.fasta_label(d), s) for d, s in O.fasta_from_lines(io.StringIO(fa, newline=None))]
    for case in g["cases"]:
        prm = case["params"]
        table = O.load_sts_lines(sts.splitlines(True), prm["wordsize"], prm["default_pcr_size"])
        lines = O.search_lines(recs, table, O.params(**prm))
        assert lines == _expected_lines(case), prm


def test_dense_repeat():
    case = load_golden("repeat.json.gz")
    table, lines = _run(case)
    assert len(lines) == case["n_hits"] == 15936
    assert lines == _expected_lines(case)


@pytest.mark.parametrize("name", ["random_cases.json.gz", "special_cases.json.gz"])
def test_random_corpus(name):
    cases = load_golden(name)["cases"]
    for i, case in enumerate(cases):
        table, lines = _run(case)
        if not case["load_ok"]:
            assert table is None, i
            continue
        assert table.max_pcr_size == case["max_pcr_size"], i
        assert len(table.records) == case["n_records"], i
        assert lines == _expected_lines(case), (i, case["params"])
        if "fasta" in case:
            fr = O.fasta_from_lines(io.StringIO(case["fasta_text"], newline=None))
            assert [[d, s] for d, s in fr] == [[d, s] for d, s, _ in case["fasta"]], i


def test_threaded_chunk_semantics():
    for case in load_golden("threaded.json.gz")["cases"]:
        table, lines = _run(case, threads=case["threads"])
        assert lines == _expected_lines(case), case["threads"]


def test_chunked_corpus():
    """-T N corpus (tests/golden/chunked.json.gz): the reference's multi-process chunking,
    duplicated overlap hits and chunk-local record ends (engine.py:380-434)."""
    for case in load_golden("chunked.json.gz")["cases"]:
        params, sts_lines, recs = case_inputs(case)
        table = O.load_sts_lines(sts_lines, params["wordsize"], params["default_pcr_size"])
        assert table.max_pcr_size == case["max_pcr_size"]
        for t, exp in case["by_threads"].items():
            lines = O.search_lines(recs, table, O.params(**params), threads=int(t))
            assert lines == exp["output"].splitlines(), (case["name"], t)


def test_oracle_hash_index_error_kats():
    """The oracle's hash restates the reference's IndexError for characters beyond U+00FF
    (errors.json.gz, generated by the reference)."""
    from oracle import epcr_oracle as O
    for p, W, exp in load_golden("errors.json.gz")["hash"]:
        try:
            got = list(O.hash_word(p, W))
        except IndexError:
            got = "IndexError"
        assert got == exp, (p, W)
