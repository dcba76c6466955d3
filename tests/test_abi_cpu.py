"""The C-ABI library loads and exports every symbol include/e2ep.h declares (CPU only;
no compute call is made without a GPU)."""
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "e2ep.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(e2ep_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = _declared()
    for must in ("e2ep_geom_index", "e2ep_lss_plan", "e2ep_lss_fwd", "e2ep_lss_bwd", "e2ep_target_bev"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from e2ep_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libe2ep_hip.so not built; run __graft_entry__.build()")
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_declared()) <= set(_lib.SIGNATURES), "ctypes table misses a declared entry point"
    assert lib.e2ep_abi_version() == 3


def test_library_is_gfx950_code_object():
    from e2ep_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
