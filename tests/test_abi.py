"""CPU: the C-ABI library loads and exports every symbol include/bsaccel.h declares."""
import ctypes
import os
import re

import pytest

from bluesky_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include', 'bsaccel.h')


def declared():
    src = open(HDR).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(bsa_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_api():
    names = declared()
    for must in ('bsa_create', 'bsa_destroy', 'bsa_set_state', 'bsa_detect', 'bsa_fetch_pairs'):
        assert must in names


def test_bindings_cover_header():
    assert sorted(_lib.SIGNATURES) == declared()


def test_library_loads_and_exports_all_symbols():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail('libbsaccel.so not built; run __graft_entry__.build()')
    raw = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared() if not hasattr(raw, n)]
    assert not missing, missing
    lib = _lib.load()
    assert lib.bsa_abi_version() == _lib.ABI_VERSION


def test_no_device_fails_loudly():
    lib = _lib.load()
    if lib.bsa_device_count() > 0:
        pytest.skip('a HIP device is visible here')
    with pytest.raises(_lib.AccelUnavailable):
        _lib.Context(0)
