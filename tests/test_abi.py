"""CPU tests: the C-ABI library loads, exports every symbol the header
declares, and its struct layouts agree with the ctypes mirror and the oracle."""
import ctypes
import os
import re

import pytest

from unpaper_hip import ctypes_abi as A
from unpaper_hip.device import EXPORTED, load_library

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "include", "unpaper_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(uphip_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_functions_listed():
    assert header_functions() == set(EXPORTED)


def test_library_exports_every_symbol():
    lib = load_library()
    missing = [n for n in EXPORTED if not hasattr(lib, n)]
    assert missing == []


@pytest.mark.parametrize("name", sorted(A.ABI_STRUCTS))
def test_struct_sizes_match(name, oracle):
    lib = load_library()
    expect = ctypes.sizeof(A.ABI_STRUCTS[name])
    assert lib.uphip_abi_sizeof(name.encode()) == expect
    assert oracle.lib.oracle_abi_sizeof(name.encode()) == expect


def test_options_defaults_agree_with_oracle(oracle):
    lib = load_library()
    a = A.Options()
    lib.uphip_options_init(ctypes.byref(a))
    b = oracle.default_options()
    assert bytes(a) == bytes(b)
    assert a.abs_black_threshold == 170 and a.abs_white_threshold == 229
    assert a.blackfilter_parameters.abs_threshold == 242
    assert a.grayfilter_parameters.abs_threshold == 127


def test_init_without_gpu_reports_status():
    lib = load_library()
    st = lib.uphip_try_init()
    assert lib.uphip_init_status_string(st)
