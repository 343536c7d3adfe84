"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of PCL 1.7 (see oracle/or_common.h header: parity vs real
PCL is unpinned).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
always as the checker, never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None
_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64 = ctypes.c_int64


def _ensure_built():
    srcs = [os.path.join(ORACLE_DIR, f) for f in os.listdir(ORACLE_DIR)
            if f.endswith((".cpp", ".h"))]
    if (not os.path.exists(ORACLE_SO)
            or max(os.path.getmtime(s) for s in srcs) > os.path.getmtime(ORACLE_SO)):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        _ensure_built()
        _lib = ctypes.CDLL(ORACLE_SO)
    return _lib


def _p(a, t=_f32p):
    return a.ctypes.data_as(t) if a is not None else None


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def radius_search(x, y, z, qx, qy, qz, r, cap=0):
    x, y, z, qx, qy, qz = map(_f32, (x, y, z, qx, qy, qz))
    nq = len(qx)
    counts = np.zeros(nq, dtype=np.int64)
    idx = d2 = None
    if cap:
        idx = np.full((nq, cap), -1, dtype=np.int32)
        d2 = np.full((nq, cap), np.nan, dtype=np.float32)
    lib().orc_radius_search(_p(x), _p(y), _p(z), _i64(len(x)), _p(qx), _p(qy), _p(qz), _i64(nq),
                            ctypes.c_double(r), _p(counts, _i64p), _p(idx, _i32p), _p(d2),
                            _i64(cap))
    return counts, idx, d2


def normals(x, y, z, r, vp=(0.0, 0.0, 0.0), threads=0):
    x, y, z = map(_f32, (x, y, z))
    n = len(x)
    out = np.empty((4, n), dtype=np.float32)
    lib().orc_normals(_p(x), _p(y), _p(z), _i64(n), ctypes.c_double(r), ctypes.c_float(vp[0]),
                      ctypes.c_float(vp[1]), ctypes.c_float(vp[2]), _p(out[0]), _p(out[1]),
                      _p(out[2]), _p(out[3]), ctypes.c_int(threads))
    return out[0], out[1], out[2], out[3]


def fpfh(sx, sy, sz, nx, ny, nz, qx, qy, qz, r, same_as_surface=False, threads=0):
    sx, sy, sz, nx, ny, nz, qx, qy, qz = map(_f32, (sx, sy, sz, nx, ny, nz, qx, qy, qz))
    nq = len(qx)
    out = np.empty((nq, 33), dtype=np.float32)
    lib().orc_fpfh(_p(sx), _p(sy), _p(sz), _p(nx), _p(ny), _p(nz), _i64(len(sx)), _p(qx), _p(qy),
                   _p(qz), _i64(nq), ctypes.c_int(1 if same_as_surface else 0),
                   ctypes.c_double(r), _p(out), ctypes.c_int(threads))
    return out
