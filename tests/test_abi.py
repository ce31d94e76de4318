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


def _reference_layout():
    import json
    with open(os.path.join(os.path.dirname(HEADER), "..", "tests", "golden",
                           "abi_layout.json")) as f:
        return json.load(f)


LAYOUT = _reference_layout()
# fields of the reference type that the HIP peer lays out identically; the
# peer's BlackfilterParameters carries its exclusions inline (the reference
# holds a pointer, filters.h:27-28), so the struct sizes differ there only
PREFIX_ONLY = {"BlackfilterParameters": "exclusions"}


@pytest.mark.parametrize("ref", sorted(LAYOUT["peers"]))
def test_layout_matches_reference_headers(ref):
    """sizeof/offsetof of every field vs the reference headers compiled by
    tests/golden/make_abi_layout.py: the adapter in INTEGRATION.md can cast
    the reference's value types to the HIP peers."""
    lib = load_library()
    peer = LAYOUT["peers"][ref].encode()
    want = LAYOUT["layout"][ref]
    for field, off in want.items():
        if field == "sizeof":
            if ref not in PREFIX_ONLY:
                assert lib.uphip_abi_sizeof(peer) == off, (ref, "sizeof")
            continue
        if PREFIX_ONLY.get(ref) == field:
            assert lib.uphip_abi_offsetof(peer, field.encode()) == off, (ref, field)
            continue
        assert lib.uphip_abi_offsetof(peer, field.encode()) == off, (ref, field)


@pytest.mark.parametrize("ref", sorted(LAYOUT["enum_peers"]))
def test_enum_sizes_match_reference(ref):
    lib = load_library()
    assert lib.uphip_abi_sizeof(LAYOUT["enum_peers"][ref].encode()) == \
        LAYOUT["layout"][ref]["sizeof"]


def test_limits_match_reference():
    import re as _re
    src = open(HEADER).read()
    assert int(_re.search(r"UPHIP_MAX_MASKS (\d+)", src).group(1)) == \
        LAYOUT["layout"]["MAX_MASKS"]["value"]
    assert int(_re.search(r"UPHIP_MAX_POINTS (\d+)", src).group(1)) == \
        LAYOUT["layout"]["MAX_POINTS"]["value"]


def test_unknown_layout_queries():
    lib = load_library()
    assert lib.uphip_abi_sizeof(b"NoSuchType") == 0
    assert lib.uphip_abi_offsetof(b"UphipPoint", b"z") == ctypes.c_size_t(-1).value
