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
    assert lib.mp_abi_version() == 2


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
