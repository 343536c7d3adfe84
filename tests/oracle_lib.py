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


def libm_mismatches(which, n, seed=0):
    """Bits where the oracle's glibc restatement differs from the host libm (0: atan2f on n
    pairs, 1: acosf on every n-th float of [-1, 1])."""
    f = lib().orc_libm_mismatches
    f.restype = ctypes.c_int64
    return int(f(ctypes.c_int(which), _i64(n), ctypes.c_uint64(seed)))


def point_covariance(x, y, z, idx):
    x, y, z = map(_f32, (x, y, z))
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    out = np.zeros(6, np.float32)
    lib().orc_point_covariance(_p(x), _p(y), _p(z), _p(idx, _i32p), _i64(len(idx)), _p(out))
    return out


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


CAM_DEFAULT = dict(width=640, height=480, center_x=320.0, center_y=240.0, focal_length_x=525.0,
                   focal_length_y=525.0, sensor_pose=np.eye(4, dtype=np.float32), coordinate_frame=0,
                   noise_level=0.0, min_range=0.0)
NARF_DEFAULT = dict(support_size=0.2, max_no_of_interest_points=-1, min_distance_between_interest_points=0.25,
                    optimal_distance_to_high_surface_change=0.25, min_interest_value=0.45,
                    min_surface_change_score=0.2, do_non_maximum_suppression=1, calculate_sparse_interest_image=1,
                    no_of_polynomial_approximations_per_point=0, add_points_on_straight_edges=0,
                    pixel_radius_borders=3, pixel_radius_plane_extraction=2, pixel_radius_border_direction=2,
                    minimum_border_probability=0.8, pixel_radius_principal_curvature=2)
_NARF_ORDER = list(NARF_DEFAULT)


def _cam(cam):
    c = dict(CAM_DEFAULT)
    c.update(cam or {})
    pose = np.ascontiguousarray(np.asarray(c["sensor_pose"], np.float32).reshape(16))
    return c, pose


def range_image_planar(x, y, z, cam=None):
    x, y, z = map(_f32, (x, y, z))
    c, pose = _cam(cam)
    out = np.empty((c["height"], c["width"], 4), dtype=np.float32)
    lib().orc_range_image_planar(_p(x), _p(y), _p(z), _i64(len(x)), ctypes.c_int(c["width"]),
                                 ctypes.c_int(c["height"]), ctypes.c_float(c["center_x"]),
                                 ctypes.c_float(c["center_y"]), ctypes.c_float(c["focal_length_x"]),
                                 ctypes.c_float(c["focal_length_y"]), _p(pose), ctypes.c_int(c["coordinate_frame"]),
                                 ctypes.c_float(c["noise_level"]), ctypes.c_float(c["min_range"]), _p(out))
    return out


def narf_keypoints(x, y, z, params=None, cam=None, debug=False, threads=0):
    x, y, z = map(_f32, (x, y, z))
    c, pose = _cam(cam)
    p = dict(NARF_DEFAULT)
    p.update(params or {})
    pv = np.array([float(p[k]) for k in _NARF_ORDER], dtype=np.float32)
    cap = c["width"] * c["height"]
    out = np.empty(cap, dtype=np.int32)
    nout = ctypes.c_int64()
    npx = c["width"] * c["height"]
    dbg_i = np.empty(npx, np.float32) if debug else None
    dbg_s = np.empty(npx, np.float32) if debug else None
    dbg_t = np.empty(npx, np.uint32) if debug else None
    lib().orc_narf_keypoints(_p(x), _p(y), _p(z), _i64(len(x)), ctypes.c_int(c["width"]), ctypes.c_int(c["height"]),
                             ctypes.c_float(c["center_x"]), ctypes.c_float(c["center_y"]),
                             ctypes.c_float(c["focal_length_x"]), ctypes.c_float(c["focal_length_y"]), _p(pose),
                             ctypes.c_int(c["coordinate_frame"]), ctypes.c_float(c["noise_level"]),
                             ctypes.c_float(c["min_range"]), _p(pv), _p(out, _i32p), _i64(cap), ctypes.byref(nout),
                             _p(dbg_i), _p(dbg_s), _p(dbg_t, ctypes.POINTER(ctypes.c_uint32)), ctypes.c_int(threads))
    kp = out[: nout.value].copy()
    if debug:
        h, w = c["height"], c["width"]
        return kp, dict(interest=dbg_i.reshape(h, w), surface_change=dbg_s.reshape(h, w),
                        border_traits=dbg_t.reshape(h, w))
    return kp


def shot(sx, sy, sz, nx, ny, nz, qx, qy, qz, r, threads=0):
    sx, sy, sz, nx, ny, nz, qx, qy, qz = map(_f32, (sx, sy, sz, nx, ny, nz, qx, qy, qz))
    nq = len(qx)
    desc = np.empty((nq, 352), dtype=np.float32)
    rf = np.empty((nq, 9), dtype=np.float32)
    lib().orc_shot(_p(sx), _p(sy), _p(sz), _p(nx), _p(ny), _p(nz), _i64(len(sx)), _p(qx), _p(qy), _p(qz), _i64(nq),
                   ctypes.c_double(r), _p(desc), _p(rf), ctypes.c_int(threads))
    return desc, rf


def nearest_descriptor(src, tgt, threads=0):
    """Features::getCorrespondences (features.h:255-273): 1-NN target row of every source row
    (-1 for a non-finite source row), and the L2_Simple squared distance."""
    src = np.ascontiguousarray(src, np.float32)
    tgt = np.ascontiguousarray(tgt, np.float32)
    ns, dim = src.shape
    idx = np.empty(ns, np.int32)
    dist = np.empty(ns, np.float32)
    rc = lib().orc_nearest_descriptor(_p(src), _i64(ns), _p(tgt), _i64(len(tgt)), ctypes.c_int(dim),
                                      _p(idx, _i32p), _p(dist), ctypes.c_int(threads))
    assert rc == 0
    return idx, dist


def correspondences(src, tgt, threads=0):
    """Features::findCorrespondences (features.h:224-253): mutual nearest neighbours as
    (index_query, index_match) arrays in source order."""
    src = np.ascontiguousarray(src, np.float32)
    tgt = np.ascontiguousarray(tgt, np.float32)
    ns, dim = src.shape
    cap = ns
    q = np.empty(cap, np.int32)
    m = np.empty(cap, np.int32)
    n = ctypes.c_int64()
    rc = lib().orc_correspondences(_p(src), _i64(ns), _p(tgt), _i64(len(tgt)), ctypes.c_int(dim), _p(q, _i32p),
                                   _p(m, _i32p), _i64(cap), ctypes.byref(n), ctypes.c_int(threads))
    assert rc == 0
    return q[: n.value].copy(), m[: n.value].copy()


_f64p = ctypes.POINTER(ctypes.c_double)


def eigen_selfadjoint3(mats):
    """Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d> eigenvalues (ascending) of (n, 3, 3)."""
    a = np.ascontiguousarray(mats, np.float64).reshape(-1, 9)
    ev = np.empty((len(a), 3), np.float64)
    assert lib().orc_eigen_selfadjoint3(_p(a, _f64p), _i64(len(a)), _p(ev, _f64p)) == 0
    return ev


def eigen_selfadjoint3_vectors(mats):
    """Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d> values (n, 3) and vectors (n, 3, 3):
    vec[i, k] = eigenvector of value k (Eigen's eigenvectors().col(k))."""
    a = np.ascontiguousarray(mats, np.float64).reshape(-1, 9)
    ev = np.empty((len(a), 3), np.float64)
    vec = np.empty((len(a), 3, 3), np.float64)
    assert lib().orc_eigen_selfadjoint3_vectors(_p(a, _f64p), _i64(len(a)), _p(ev, _f64p), _p(vec, _f64p)) == 0
    return ev, vec


def cloud_resolution(x, y, z, threads=0):
    """Keypoints::computeCloudResolution (keypoints.h:401-428): (resolution, per-point terms)."""
    x, y, z = map(_f32, (x, y, z))
    out = ctypes.c_double()
    terms = np.empty(len(x), np.float32)
    assert lib().orc_cloud_resolution(_p(x), _p(y), _p(z), _i64(len(x)), ctypes.byref(out), _p(terms),
                                      ctypes.c_int(threads)) == 0
    return out.value, terms


def iss_keypoints(x, y, z, salient_radius, non_max_radius, min_neighbors=5, gamma21=0.975, gamma32=0.975,
                  threads=0):
    """ISSKeypoint3D::compute (PCL 1.7) as keypoints.h:177-189 configures it: (indices, third)."""
    x, y, z = map(_f32, (x, y, z))
    n = len(x)
    idx = np.empty(max(n, 1), np.int32)
    third = np.empty(n, np.float64)
    k = ctypes.c_int64()
    rc = lib().orc_iss_keypoints(_p(x), _p(y), _p(z), _i64(n), ctypes.c_double(salient_radius),
                                 ctypes.c_double(non_max_radius), ctypes.c_int(min_neighbors),
                                 ctypes.c_double(gamma21), ctypes.c_double(gamma32), _p(idx, _i32p), _i64(len(idx)),
                                 ctypes.byref(k), _p(third, _f64p), ctypes.c_int(threads))
    if rc == 1:
        return np.empty(0, np.int32), np.zeros(n)
    assert rc == 0, rc
    return idx[: k.value].copy(), third


def harris3d(x, y, z, radius=0.01, threshold=1e-6, refine=True, threads=0):
    """HarrisKeypoint3D (keypoints.h:150-162) + getKeypointsCloud (keypoints.h:365-395):
    (snapped cloud indices, per-point response, refined corners (nc, 3))."""
    x, y, z = map(_f32, (x, y, z))
    n = len(x)
    cap = max(n, 1)
    idx = np.empty(cap, np.int32)
    resp = np.empty(max(n, 1), np.float32)
    corners = np.empty((cap, 3), np.float32)
    k, nc = ctypes.c_int64(), ctypes.c_int64()
    rc = lib().orc_harris3d(_p(x), _p(y), _p(z), _i64(n), ctypes.c_double(radius), ctypes.c_float(threshold),
                            ctypes.c_int(1 if refine else 0), _p(idx, _i32p), _i64(cap), ctypes.byref(k),
                            ctypes.byref(nc), _p(resp), _p(corners), ctypes.c_int(threads))
    assert rc == 0, rc
    return idx[: k.value].copy(), resp[:n].copy(), corners[: nc.value].copy()


def harris6d(x, y, z, rgb, radius=0.01, threshold=1e-6, refine=True, threads=0):
    """HarrisKeypoint6D (keypoints.h:164-176) + getKeypointsCloud (keypoints.h:365-395):
    (snapped cloud indices, per-point response, refined corners (nc, 3), normalised intensity
    gradients (n, 3)).  rgb: packed 0x00RRGGBB."""
    x, y, z = map(_f32, (x, y, z))
    rgb = np.ascontiguousarray(rgb, dtype=np.uint32)
    n = len(x)
    cap = max(n, 1)
    idx = np.empty(cap, np.int32)
    resp = np.empty(max(n, 1), np.float32)
    corners = np.empty((cap, 3), np.float32)
    grad = np.empty((max(n, 1), 3), np.float32)
    k, nc = ctypes.c_int64(), ctypes.c_int64()
    rc = lib().orc_harris6d(_p(x), _p(y), _p(z), _p(rgb, ctypes.POINTER(ctypes.c_uint32)), _i64(n),
                            ctypes.c_double(radius), ctypes.c_float(threshold), ctypes.c_int(1 if refine else 0),
                            _p(idx, _i32p), _i64(cap), ctypes.byref(k), ctypes.byref(nc), _p(resp), _p(corners),
                            _p(grad), ctypes.c_int(threads))
    assert rc == 0, rc
    return idx[: k.value].copy(), resp[:n].copy(), corners[: nc.value].copy(), grad[:n].copy()


def eigen_selfadjoint6f(a):
    """Eigen 3.2 SelfAdjointEigenSolver<Matrix<float,6,6>> eigenvalues of (m, 6, 6) float32
    matrices (lower triangle read); returns (ev (m, 6), count of non-converged)."""
    a = np.ascontiguousarray(np.asarray(a, np.float32).transpose(0, 2, 1))  # column-major
    m = a.shape[0]
    ev = np.empty((m, 6), np.float32)
    bad = lib().orc_eigen_selfadjoint6f(_p(a), _i64(m), _p(ev))
    return ev, bad


def colpiv_solve3f(a, b):
    """Eigen 3.2 ColPivHouseholderQR<Matrix3f>(a).solve(b) for (m, 3, 3) / (m, 3) float32."""
    a = np.ascontiguousarray(np.asarray(a, np.float32).transpose(0, 2, 1))
    b = np.ascontiguousarray(b, np.float32)
    x = np.empty_like(b)
    lib().orc_colpiv_solve3f(_p(a), _p(b), _i64(a.shape[0]), _p(x))
    return x


def u8_cast(v, native=False):
    """static_cast<uint8_t>(float) as the restatement models it (native=True: the host g++'s
    own code for the cast, the pin of the model)."""
    v = _f32(v)
    out = np.empty(len(v), np.int32)
    f = lib().orc_u8_cast_native if native else lib().orc_u8_cast_model
    f(_p(v), _i64(len(v)), _p(out, _i32p))
    return out


def ransac_rejector(src, tgt, query, match, threshold=0.015, max_iterations=1000):
    """Features::filterCorrespondences (features.h:282-297): (kept correspondence positions,
    4x4 best transformation, models evaluated).  src / tgt: (n, 3) keypoint clouds."""
    src = np.ascontiguousarray(src, np.float32)
    tgt = np.ascontiguousarray(tgt, np.float32)
    sx, sy, sz = (np.ascontiguousarray(src[:, i]) for i in range(3))
    tx, ty, tz = (np.ascontiguousarray(tgt[:, i]) for i in range(3))
    query = np.ascontiguousarray(query, np.int32)
    match = np.ascontiguousarray(match, np.int32)
    n = len(query)
    keep = np.empty(max(n, 1), np.int32)
    nk, it = ctypes.c_int64(), ctypes.c_int64()
    T = np.empty(16, np.float32)
    assert lib().orc_ransac_rejector(_p(sx), _p(sy), _p(sz), _i64(len(sx)), _p(tx), _p(ty), _p(tz), _i64(len(tx)),
                                     _p(query, _i32p), _p(match, _i32p), _i64(n), ctypes.c_double(threshold),
                                     ctypes.c_int(max_iterations), _p(keep, _i32p), ctypes.byref(nk), _p(T),
                                     ctypes.byref(it)) == 0
    return keep[: nk.value].copy(), T.reshape(4, 4), it.value
