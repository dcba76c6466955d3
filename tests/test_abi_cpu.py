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
    assert lib.e2ep_abi_version() == 4


def test_library_is_gfx950_code_object():
    from e2ep_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_dwconv_bf16_predicate_host_only():
    """e2ep_dwconv_bf16_ok is a host-side geometry predicate (no GPU call): the MBConv
    depthwise shapes of the C3 step take bf16 storage, geometries without a strip kernel or with
    planes not a multiple of 4 do not.  dims = (N, C, H, W, K, P, Q, stride, pad_top, pad_left)."""
    import ctypes
    from e2ep_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libe2ep_hip.so not built; run __graft_entry__.build()")
    lib = _lib.load()

    def ok(*d):
        return lib.e2ep_dwconv_bf16_ok((ctypes.c_int * 10)(*d))

    assert ok(32, 192, 64, 64, 3, 64, 64, 1, 1, 1) == 1     # k3 s1
    assert ok(32, 336, 32, 32, 5, 32, 32, 1, 2, 2) == 1     # k5 s1
    assert ok(32, 144, 128, 128, 3, 64, 64, 2, 0, 0) == 1   # k3 s2
    assert ok(2, 32, 30, 30, 3, 30, 30, 1, 1, 1) == 0       # W % 4 != 0
    assert ok(2, 16, 16, 16, 7, 16, 16, 1, 3, 3) == 0       # K = 7
    assert ok(2, 32, 18, 18, 5, 9, 9, 2, 2, 2) == 0         # 9 x 9 output
    assert ok(0, 32, 16, 16, 3, 16, 16, 1, 1, 1) == 0       # empty batch
