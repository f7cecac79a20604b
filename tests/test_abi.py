"""The C-ABI library builds, loads and exports every symbol include/merpcr_hip.h declares.

No compute calls here (CPU container); on a host without a GPU the entry
points must fail loudly rather than fall back to CPU code.
"""

import ctypes
import os
import re

import pytest

from merpcr_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "merpcr_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|int32_t|const char\*)\s+(mp_\w+)\(", text, re.M)))


def test_header_and_binding_agree():
    assert _declared() == sorted(_native.EXPORTS)


def test_library_exports_all_symbols():
    lib = _native.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.mp_abi_version() == _native.ABI_VERSION == 3


_LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "merpcr_hip.h"
#define F(T, f) printf("%s.%s %zu %zu\n", #T, #f, offsetof(T, f), sizeof(((T*)0)->f));
int main(void) {
    printf("mp_search_options %zu\n", sizeof(mp_search_options));
    printf("mp_table_options %zu\n", sizeof(mp_table_options));
    F(mp_search_options, tails) F(mp_search_options, no_defer) F(mp_search_options, no_dense)
    F(mp_search_options, sort) F(mp_search_options, sort_bucket_bits) F(mp_search_options, pair_blocks_per_cu)
    F(mp_search_options, hit_cap) F(mp_search_options, surv_cap) F(mp_search_options, tail_cap)
    F(mp_search_options, no_rank_filter) F(mp_search_options, no_split) F(mp_search_options, generic_forms)
    F(mp_search_options, ref32) F(mp_search_options, sched_short) F(mp_search_options, crowd_grid) F(mp_search_options, scan_grid)
    F(mp_table_options, lds_k) F(mp_table_options, no_h12) F(mp_table_options, kgrp4) F(mp_table_options, no_split)
    printf("MP_GENERIC %u %u %u\n", MP_GENERIC_FIX, MP_GENERIC_GAP, MP_GENERIC_PAIR);
    printf("MP_GATHER %d %d\n", MP_GATHER_COPY, MP_GATHER_RCCL);
    printf("MP_LAYOUT %u %u %u %u %u %u %u %u\n", MP_LAYOUT_LDS_EXACT, MP_LAYOUT_RANK, MP_LAYOUT_KGRP, MP_LAYOUT_KGRP4,
           MP_LAYOUT_DENSE, MP_LAYOUT_SPLIT, MP_LAYOUT_HASHED, MP_LAYOUT_DEFER_FULL);
    return 0;
}
"""


def test_option_structs_match_the_header(tmp_path):
    """The ctypes mirrors of mp_search_options / mp_table_options and the option constants
    have the header's layout (compiled with the host C compiler against include/)."""
    import subprocess
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    rows = dict((ln.split(" ", 1)[0], ln.split(" ", 1)[1]) for ln in out if ln)
    for name, cls in (("mp_search_options", _native.MPSearchOptions), ("mp_table_options", _native.MPTableOptions)):
        assert int(rows[name]) == ctypes.sizeof(cls), name
        for f, _ in cls._fields_:
            off, size = map(int, rows[f"{name}.{f}"].split())
            assert (getattr(cls, f).offset, getattr(cls, f).size) == (off, size), (name, f)
    assert [int(x) for x in rows["MP_GENERIC"].split()] == [_native.MP_GENERIC[k] for k in ("fix", "gap", "pair")]
    assert [int(x) for x in rows["MP_GATHER"].split()] == [_native.MP_GATHER[k] for k in ("copy", "rccl")]
    assert [int(x) for x in rows["MP_LAYOUT"].split()] == list(_native.Table.LAYOUT.values())


def test_table_options_out_of_range_is_value_error():
    """mp_table_create_ex checks its options before touching a device."""
    prm = _native.MPParams(11, 50, 0, 1, 0)
    with pytest.raises(ValueError):
        _native.Table(prm, 0, [], [], [], b"", [0], b"", [0], lds_k=4)


def test_device_count_and_loud_failure_without_gpu():
    n = _native.device_count()
    if n > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    prm = _native.MPParams(11, 50, 0, 1, 0)
    with pytest.raises(Exception):
        _native.Table(prm, 0, [], [], [], b"", [0], b"", [0])
    from merpcr_amd import FASTARecord, MerPCR
    eng = MerPCR()
    with pytest.raises(Exception):
        eng.find_hits([FASTARecord(defline=">x", sequence="ACGT" * 10)])


def test_bad_params_map_to_value_error():
    prm = _native.MPParams(2, 50, 0, 1, 0)  # W below the reference's bound
    with pytest.raises(ValueError):
        _native.Table(prm, 0, [], [], [], b"", [0], b"", [0])
