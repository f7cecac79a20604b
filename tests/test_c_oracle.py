"""Pin the C oracle (oracle/epcr_oracle.c) against the reference's golden outputs."""

import pytest

from oracle import c_oracle as C
from oracle import epcr_oracle as O
from tests.golden_io import case_inputs, load_golden


def _lines(case, nthreads=1):
    params, sts_lines, recs = case_inputs(case)
    table = O.load_sts_lines(sts_lines, params["wordsize"], params["default_pcr_size"])
    if table is None:
        return None
    return C.lines(table, recs, O.params(**params), nthreads)


@pytest.mark.parametrize("nthreads", [1, 3])
def test_c_oracle_golden(nthreads):
    for name in ("random_cases.json.gz", "special_cases.json.gz"):
        for i, case in enumerate(load_golden(name)["cases"]):
            got = _lines(case, nthreads)
            if not case["load_ok"]:
                assert got is None
                continue
            # the golden corpus is ASCII except the FASTA long-s case, which upper-cases to ASCII
            assert got == case["output"].splitlines(), (name, i)


def test_c_oracle_repeat():
    case = load_golden("repeat.json.gz")
    assert _lines(case, 4) == case["output"].splitlines()


def test_c_oracle_threaded_case_t1():
    case = load_golden("threaded.json.gz")["cases"][0]
    assert case["threads"] == 1
    assert _lines(case, 5) == case["output"].splitlines()
