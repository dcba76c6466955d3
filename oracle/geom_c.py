"""ORACLE / TEST INFRASTRUCTURE ONLY — ctypes wrapper of the plain-C pillar-index oracle."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle_geom.so")


def _lib():
    if not os.path.exists(_SO):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    lib = ctypes.CDLL(_SO)
    lib.oracle_geom_index.restype = None
    return lib


def geom_index(frustum, combine, trans, lo, res, dims, with_xyz=False):
    """frustum (D,h,w,3), combine (B*N,3,3), trans (B*N,3) float32 arrays -> int32 pillar
    (B*N, D, h, w) [and xyz (B*N, D, h, w, 3)]."""
    fr = np.ascontiguousarray(frustum, np.float32)
    cb = np.ascontiguousarray(combine, np.float32).reshape(-1, 3, 3)
    tr = np.ascontiguousarray(trans, np.float32).reshape(-1, 3)
    lo = np.ascontiguousarray(lo, np.float32)
    res = np.ascontiguousarray(res, np.float32)
    D, h, w, _ = fr.shape
    BN = cb.shape[0]
    out = np.empty((BN, D, h, w), np.int32)
    xyz = np.empty((BN, D, h, w, 3), np.float32) if with_xyz else None
    P = ctypes.c_void_p
    _lib().oracle_geom_index(
        fr.ctypes.data_as(P), cb.ctypes.data_as(P), tr.ctypes.data_as(P), lo.ctypes.data_as(P),
        res.ctypes.data_as(P), int(dims[0]), int(dims[1]), int(dims[2]), 1, BN, D, h, w,
        out.ctypes.data_as(P), xyz.ctypes.data_as(P) if with_xyz else None)
    return (out, xyz) if with_xyz else out
