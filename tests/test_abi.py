"""The C-ABI library loads and exports every symbol include/psg.h declares.

CPU-only: host-side entry points (server ranges, argument validation) are
called; nothing that launches a kernel.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
import psg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "psg.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(psg_\w+)\s*\(", text, re.M)))


def test_header_declares_what_binding_binds():
    assert declared_symbols() == sorted(psg.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", psg.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (psg_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = psg.lib()
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_abi_version():
    assert psg.lib().psg_abi_version() == 1


def test_server_ranges_match_oracle():
    for ns in (1, 2, 3, 5, 8, 64):
        b, e = psg.server_ranges(ns)
        ob, oe = oracle.server_ranges(ns)
        np.testing.assert_array_equal(b, ob)
        np.testing.assert_array_equal(e, oe)


def test_invalid_arguments_fail_loudly():
    with pytest.raises(psg.PsgError) as ei:
        psg.Store(7, psg.F32, 0, 10, 10)  # bad kind, rejected before any HIP call
    assert ei.value.code == 1 and "bad kind" in str(ei.value)
    with pytest.raises(psg.PsgError):
        psg.Store(psg.DENSE, 99, 0, 10, 10)  # bad dtype
    with pytest.raises(psg.PsgError):
        psg.Store(psg.DENSE, psg.F32, 0, 10, 11)  # capacity beyond the key range
    # merge whose replies do not add up ("lost some servers?", KVApp.h:691)
    with pytest.raises(psg.PsgError) as ei:
        psg.merge([(0x1000, 3, 0)], 4, 0x2000, 4)
    assert "lost some servers" in str(ei.value)
    # slicer with non-adjacent ranges (KVApp.h:531)
    b, e = psg.server_ranges(2)
    e[0] -= 1
    with pytest.raises(psg.PsgError):
        psg.slice_keys(0x1000, 4, b, e)


def test_empty_requests_are_noops():
    b, e = psg.server_ranges(3)
    kp, vp = psg.slice_keys(None, 0, b, e)
    assert kp.tolist() == [0, 0, 0, 0] and vp.tolist() == [0, 0, 0, 0]
    psg.merge([], 4, None, 0)


def test_oracle_library_loads():
    assert oracle.lib() is not None
