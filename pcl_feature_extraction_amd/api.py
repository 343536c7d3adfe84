"""Python front-end of libpfx (host numpy arrays or torch device tensors).

Every call goes through the HIP C-ABI (include/pfx.h); nothing here computes features on the
CPU.  ``Context`` owns one ``pfx_ctx`` (one HIP stream) on one device.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(a.data_ptr())  # torch tensor (device pointer)


def narf_params(support_size=0.2, **kw) -> N.NarfParams:
    p = N.NarfParams()
    N.lib().pfx_narf_params_default(ctypes.byref(p))
    p.support_size = support_size
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def pcd_header(path) -> N.PcdHeader:
    """PCD header through the C-ABI (host only: no device needed)."""
    h = N.PcdHeader()
    st = N.lib().pfx_pcd_read_header(str(path).encode(), ctypes.byref(h))
    if st != 0:
        raise N.PfxError(st, f"pfx_pcd_read_header({path})")
    return h


def camera(**kw) -> N.Camera:
    c = N.Camera()
    N.lib().pfx_camera_default(ctypes.byref(c))
    for k, v in kw.items():
        if k == "sensor_pose":
            for i, e in enumerate(np.asarray(v, dtype=np.float32).reshape(16)):
                c.sensor_pose[i] = float(e)
        else:
            setattr(c, k, v)
    return c


class Context:
    def __init__(self, device: int = 0):
        self._lib = N.lib()
        h = ctypes.c_void_p()
        code = self._lib.pfx_ctx_create(device, ctypes.byref(h))
        if code != 0:
            raise N.PfxError(code, f"pfx_ctx_create(device={device}) failed")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self._lib.pfx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, code):
        if code != 0:
            raise N.PfxError(code, self._lib.pfx_last_error(self.h).decode())

    # ---- plumbing ------------------------------------------------------------------
    def set_stream(self, stream_handle):
        """Run on an external HIP stream (torch's `stream.cuda_stream`; 0 = the null stream)."""
        self._check(self._lib.pfx_ctx_set_stream(self.h, ctypes.c_void_p(stream_handle)))

    def use_own_stream(self):
        self._check(self._lib.pfx_ctx_use_own_stream(self.h))

    def synchronize(self):
        """Waits for this context's stream; raises deferred errors of the stream-ordered calls
        (an FPFH neighbourhood beyond capacity -> PfxError, its rows NaN)."""
        self._check(self._lib.pfx_ctx_synchronize(self.h))

    def trim(self):
        """Frees every device scratch buffer of this context (pfx_ctx_trim)."""
        self._check(self._lib.pfx_ctx_trim(self.h))

    def set_shared(self, shared=True):
        """Launch-shape hint: another stream runs latency-critical work on this device
        concurrently (pfx_ctx_set_shared); results are unchanged."""
        self._check(self._lib.pfx_ctx_set_shared(self.h, 1 if shared else 0))

    def set_timing(self, enable=True, stages_only=False):
        """HIP-event timers on this context's stream: every kernel group, or (stages_only) one event
        pair per stage call (normals, normals_fast, shot, iss, ...: the live roofline's timer)."""
        self._check(self._lib.pfx_ctx_set_timing(self.h, (2 if stages_only else 1) if enable else 0))

    def reset_timing(self):
        self._check(self._lib.pfx_ctx_reset_timing(self.h))

    def kernel_time(self, name):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        self._check(self._lib.pfx_ctx_kernel_time(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def stat(self, name):
        v = ctypes.c_int64()
        self._check(self._lib.pfx_ctx_last_stats(self.h, name.encode(), ctypes.byref(v)))
        return v.value

    # ---- host-array entry points ---------------------------------------------------
    def radius_search(self, x, y, z, qx, qy, qz, r, cap=0):
        x, y, z, qx, qy, qz = map(_f32, (x, y, z, qx, qy, qz))
        nq = len(qx)
        counts = np.zeros(nq, dtype=np.int64)
        idx = d2 = None
        if cap:
            idx = np.full((nq, cap), -1, dtype=np.int32)
            d2 = np.full((nq, cap), np.nan, dtype=np.float32)
        self._check(self._lib.pfx_radius_search(self.h, _ptr(x), _ptr(y), _ptr(z), len(x), _ptr(qx), _ptr(qy),
                                                _ptr(qz), nq, float(r), _ptr(counts), _ptr(idx), _ptr(d2),
                                                int(cap)))
        return counts, idx, d2

    def normals(self, x, y, z, r, viewpoint=(0.0, 0.0, 0.0)):
        x, y, z = map(_f32, (x, y, z))
        n = len(x)
        out = np.empty((4, n), dtype=np.float32)
        vp = _f32(viewpoint)
        self._check(self._lib.pfx_normals(self.h, _ptr(x), _ptr(y), _ptr(z), n, float(r), _ptr(vp), _ptr(out[0]),
                                          _ptr(out[1]), _ptr(out[2]), _ptr(out[3])))
        return out[0], out[1], out[2], out[3]

    def normals_fast(self, x, y, z, r, viewpoint=(0.0, 0.0, 0.0)):
        """Opt-in MFMA-covariance normals (pfx_normals_fast): not parity-exact, see include/pfx.h."""
        x, y, z = map(_f32, (x, y, z))
        n = len(x)
        out = np.empty((4, n), dtype=np.float32)
        vp = _f32(viewpoint)
        self._check(self._lib.pfx_normals_fast(self.h, _ptr(x), _ptr(y), _ptr(z), n, float(r), _ptr(vp),
                                               _ptr(out[0]), _ptr(out[1]), _ptr(out[2]), _ptr(out[3])))
        return out[0], out[1], out[2], out[3]

    def fpfh(self, sx, sy, sz, nx, ny, nz, qx, qy, qz, r, same_as_surface=False):
        sx, sy, sz, nx, ny, nz = map(_f32, (sx, sy, sz, nx, ny, nz))
        if same_as_surface:
            qx, qy, qz = sx, sy, sz
        qx, qy, qz = map(_f32, (qx, qy, qz))
        nq = len(qx)
        out = np.empty((nq, 33), dtype=np.float32)
        self._check(self._lib.pfx_fpfh(self.h, _ptr(sx), _ptr(sy), _ptr(sz), _ptr(nx), _ptr(ny), _ptr(nz), len(sx),
                                       _ptr(qx), _ptr(qy), _ptr(qz), nq, 1 if same_as_surface else 0, float(r),
                                       _ptr(out)))
        return out

    def shot(self, sx, sy, sz, nx, ny, nz, qx, qy, qz, r):
        sx, sy, sz, nx, ny, nz, qx, qy, qz = map(_f32, (sx, sy, sz, nx, ny, nz, qx, qy, qz))
        nq = len(qx)
        desc = np.empty((nq, 352), dtype=np.float32)
        rf = np.empty((nq, 9), dtype=np.float32)
        self._check(self._lib.pfx_shot(self.h, _ptr(sx), _ptr(sy), _ptr(sz), _ptr(nx), _ptr(ny), _ptr(nz), len(sx),
                                       _ptr(qx), _ptr(qy), _ptr(qz), nq, float(r), _ptr(desc), _ptr(rf)))
        return desc, rf

    def range_image_planar(self, x, y, z, cam=None):
        cam = cam or camera()
        x, y, z = map(_f32, (x, y, z))
        out = np.empty((cam.height, cam.width, 4), dtype=np.float32)
        self._check(self._lib.pfx_range_image_planar(self.h, _ptr(x), _ptr(y), _ptr(z), len(x), ctypes.byref(cam),
                                                     _ptr(out)))
        return out

    def narf_keypoints(self, x, y, z, params=None, cam=None, cap=1 << 20):
        cam = cam or camera()
        params = params or narf_params()
        x, y, z = map(_f32, (x, y, z))
        out = np.empty(cap, dtype=np.int32)
        nout = ctypes.c_int64()
        self._check(self._lib.pfx_narf_keypoints(self.h, _ptr(x), _ptr(y), _ptr(z), len(x), ctypes.byref(cam),
                                                 ctypes.byref(params), _ptr(out), cap, ctypes.byref(nout)))
        return out[: nout.value].copy()

    def narf_debug_image(self, which, width=640, height=480):
        dt = np.uint32 if which == "border_traits" else np.float32
        out = np.empty(width * height, dtype=dt)
        self._check(self._lib.pfx_narf_debug_image(self.h, which.encode(), _ptr(out), out.size))
        return out.reshape(height, width)

    # ---- device (torch tensor) entry points, stream-ordered on the ctx stream ---------
    def normals_dev(self, x, y, z, r, nx, ny, nz, curv, viewpoint=(0.0, 0.0, 0.0)):
        vp = _f32(viewpoint)
        self._check(self._lib.pfx_normals_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r), _ptr(vp),
                                              _ptr(nx), _ptr(ny), _ptr(nz), _ptr(curv)))

    def normals_fast_dev(self, x, y, z, r, nx, ny, nz, curv, viewpoint=(0.0, 0.0, 0.0)):
        vp = _f32(viewpoint)
        self._check(self._lib.pfx_normals_fast_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r), _ptr(vp),
                                                   _ptr(nx), _ptr(ny), _ptr(nz), _ptr(curv)))

    def fpfh_dev(self, sx, sy, sz, nx, ny, nz, qx, qy, qz, r, out, same_as_surface=False, after_normals=False):
        """after_normals: the caller vouches that (sx, sy, sz) still hold the cloud of this context's
        last normals_dev (Features::compute's sequence) -> pfx_fpfh_after_normals_dev, which may
        reuse that estimation's neighbour lists."""
        fn = self._lib.pfx_fpfh_after_normals_dev if after_normals else self._lib.pfx_fpfh_dev
        self._check(fn(self.h, _ptr(sx), _ptr(sy), _ptr(sz), _ptr(nx), _ptr(ny), _ptr(nz), sx.numel(), _ptr(qx),
                       _ptr(qy), _ptr(qz), qx.numel(), 1 if same_as_surface else 0, float(r), _ptr(out)))

    def normals_lists_dev(self, x, y, z, r, nx, ny, nz, curv):
        """Phase 1 of normals_dev: neighbour lists of every point (kept in this context)."""
        self._check(self._lib.pfx_normals_lists_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r), _ptr(nx),
                                                    _ptr(ny), _ptr(nz), _ptr(curv)))

    def normals_launch_dev(self, x, y, z, r, nx, ny, nz, curv, viewpoint=(0.0, 0.0, 0.0)):
        """normals_dev with no host round trip (pfx_normals_launch_dev); normals_finish_dev must
        follow before the outputs are trusted."""
        vp = (ctypes.c_float * 3)(*viewpoint)
        self._check(self._lib.pfx_normals_launch_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r), vp,
                                                     _ptr(nx), _ptr(ny), _ptr(nz), _ptr(curv)))

    def normals_grid_launch_dev(self, x, y, z, r):
        """Queue the spatial grid of the next normals_launch_dev on this context's stream now
        (pfx_normals_grid_launch_dev) so it runs ahead of work issued later on other streams;
        the launch for the same cloud and radius then starts at its list kernels."""
        self._check(self._lib.pfx_normals_grid_launch_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r)))

    def normals_gate_dev(self, event):
        """The next normals launch on this context waits for `event` (a recorded torch.cuda.Event)
        between its grid build and its list kernels (pfx_normals_gate_dev); None clears it."""
        self._check(self._lib.pfx_normals_gate_dev(self.h, None if event is None else event.cuda_event))

    def normals_finish_dev(self) -> bool:
        """Validates the launched estimation; True when it had to be rerun (consumers of its
        outputs queued in between must run again)."""
        rerun = ctypes.c_int32(0)
        self._check(self._lib.pfx_normals_finish_dev(self.h, ctypes.byref(rerun)))
        return bool(rerun.value)

    def normals_prepare_dev(self, x, y, z, r):
        """The grid of the next normals_subset_dev calls on this cloud, built ahead (coordinates only)."""
        self._check(self._lib.pfx_normals_prepare_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r)))

    def normals_subset_dev(self, x, y, z, r, mask, want, nx, ny, nz, curv, viewpoint=(0.0, 0.0, 0.0)):
        """NormalEstimationOMP for the points with (mask != 0) == want only (uint8 device mask by
        point); the other output entries are left untouched."""
        vp = (ctypes.c_float * 3)(*viewpoint)
        self._check(self._lib.pfx_normals_subset_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), float(r),
                                                     _ptr(mask), int(want), vp, _ptr(nx), _ptr(ny), _ptr(nz),
                                                     _ptr(curv)))

    def normals_chains_dev(self, lists_ctx, nx, ny, nz, curv, mask=None, want=1, viewpoint=(0.0, 0.0, 0.0)):
        """Phase 2 on this context's stream for the points with (mask != 0) == want (all if mask
        is None), from the lists held by `lists_ctx`."""
        vp = (ctypes.c_float * 3)(*viewpoint)
        self._check(self._lib.pfx_normals_chains_dev(self.h, lists_ctx.h, _ptr(mask), int(want), vp, _ptr(nx),
                                                     _ptr(ny), _ptr(nz), _ptr(curv)))

    def fpfh_support_mask_dev(self, sx, sy, sz, qx, qy, qz, r, mask):
        """mask[i] = 1 for the surface points FPFH reads normals of (within r of a query)."""
        self._check(self._lib.pfx_fpfh_support_mask_dev(self.h, _ptr(sx), _ptr(sy), _ptr(sz), sx.numel(), _ptr(qx),
                                                         _ptr(qy), _ptr(qz), qx.numel(), float(r), _ptr(mask)))

    def fpfh_support_ball_dev(self, sx, sy, sz, qx, qy, qz, r, mask):
        """Conservative support: mask[i] = 1 for the surface points within 2r of a query."""
        self._check(self._lib.pfx_fpfh_support_ball_dev(self.h, _ptr(sx), _ptr(sy), _ptr(sz), sx.numel(), _ptr(qx),
                                                         _ptr(qy), _ptr(qz), qx.numel(), float(r), _ptr(mask)))

    def fpfh_prepare_queries_dev(self, sx, sy, sz, qx, qy, qz, r):
        """The next fpfh_dev's SPFH point set for these queries (same tensors), found ahead."""
        self._check(self._lib.pfx_fpfh_prepare_queries_dev(self.h, _ptr(sx), _ptr(sy), _ptr(sz), sx.numel(),
                                                            _ptr(qx), _ptr(qy), _ptr(qz), qx.numel(), float(r)))

    def fpfh_prepare_dev(self, sx, sy, sz, r):
        """Build the FPFH search-surface index ahead of fpfh_dev (see pfx_fpfh_prepare_dev)."""
        self._check(self._lib.pfx_fpfh_prepare_dev(self.h, _ptr(sx), _ptr(sy), _ptr(sz), sx.numel(), float(r)))

    def shot_dev(self, sx, sy, sz, nx, ny, nz, qx, qy, qz, r, desc, rf):
        self._check(self._lib.pfx_shot_dev(self.h, _ptr(sx), _ptr(sy), _ptr(sz), _ptr(nx), _ptr(ny), _ptr(nz),
                                           sx.numel(), _ptr(qx), _ptr(qy), _ptr(qz), qx.numel(), float(r),
                                           _ptr(desc), _ptr(rf)))

    def narf_keypoints_dev(self, x, y, z, params=None, cam=None, cap=1 << 20):
        cam = cam or camera()
        params = params or narf_params()
        out = np.empty(cap, dtype=np.int32)
        nout = ctypes.c_int64()
        self._check(self._lib.pfx_narf_keypoints_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(),
                                                     ctypes.byref(cam), ctypes.byref(params), _ptr(out), cap,
                                                     ctypes.byref(nout)))
        return out[: nout.value].copy()

    def gather_points_dev(self, x, y, z, idx_np, kx, ky, kz):
        idx = np.ascontiguousarray(idx_np, dtype=np.int32)
        nout = ctypes.c_int64()
        self._check(self._lib.pfx_gather_points_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), _ptr(idx),
                                                    len(idx), _ptr(kx), _ptr(ky), _ptr(kz),
                                                    min(kx.numel(), ky.numel(), kz.numel()), ctypes.byref(nout)))
        return nout.value

    # ---- PCD input: pcl::io::loadPCDFile<PointXYZRGB> (evaluation.cpp:226-235) -------------
    def pcd_load_xyz_dev(self, path, x, y, z):
        """x, y, z (float32 device tensors of >= POINTS elements) <- the file's points; returns
        (n, header)."""
        n = ctypes.c_int64()
        h = N.PcdHeader()
        self._check(self._lib.pfx_pcd_load_xyz_dev(self.h, str(path).encode(), _ptr(x), _ptr(y), _ptr(z), x.numel(),
                                                   ctypes.byref(n), ctypes.byref(h)))
        return n.value, h

    # ---- descriptor matching: Features<T>::findCorrespondences / getCorrespondences ----------
    def correspondences(self, src, tgt):
        """features.h:224-253: mutual nearest neighbours (index_query, index_match) in source
        order; src / tgt are (n, D) float32 descriptor matrices (host)."""
        src = np.ascontiguousarray(src, dtype=np.float32)
        tgt = np.ascontiguousarray(tgt, dtype=np.float32)
        ns, d = src.shape
        q = np.empty(max(ns, 1), np.int32)
        m = np.empty(max(ns, 1), np.int32)
        n = ctypes.c_int64()
        self._check(self._lib.pfx_correspondences(self.h, _ptr(src), ns, d, _ptr(tgt), tgt.shape[0], tgt.shape[1], d,
                                                  _ptr(q), _ptr(m), ns, ctypes.byref(n)))
        return q[: n.value].copy(), m[: n.value].copy()

    def nearest_descriptors(self, src, tgt):
        """features.h:255-273 (one direction, host arrays): nearest target row of every source row
        (-1: non-finite row / empty target) and its L2_Simple squared distance."""
        src = np.ascontiguousarray(src, dtype=np.float32)
        tgt = np.ascontiguousarray(tgt, dtype=np.float32)
        ns, d = src.shape
        idx = np.empty(max(ns, 1), np.int32)
        dist = np.empty(max(ns, 1), np.float32)
        self._check(self._lib.pfx_nearest_descriptors(self.h, _ptr(src), ns, d, _ptr(tgt), tgt.shape[0], tgt.shape[1],
                                                      d, _ptr(idx), _ptr(dist)))
        return idx[:ns].copy(), dist[:ns].copy()

    def nearest_descriptors_dev(self, src, tgt, s2t, s2t_dist=None, t2s=None, t2s_dist=None, dim=None):
        """features.h:255-273 in both directions: (n, stride) device tensors, `dim` leading floats
        of each row compared (default: the whole row)."""
        dim = dim or src.shape[1]
        self._check(self._lib.pfx_nearest_descriptors_dev(self.h, _ptr(src), src.shape[0], src.stride(0),
                                                          _ptr(tgt), tgt.shape[0], tgt.stride(0), dim, _ptr(s2t),
                                                          _ptr(s2t_dist), _ptr(t2s), _ptr(t2s_dist)))

    def correspondences_dev(self, src, tgt, query, match, dim=None):
        """Device version of correspondences(); returns the number of pairs written."""
        dim = dim or src.shape[1]
        n = ctypes.c_int64()
        self._check(self._lib.pfx_correspondences_dev(self.h, _ptr(src), src.shape[0], src.stride(0), _ptr(tgt),
                                                      tgt.shape[0], tgt.stride(0), dim, _ptr(query), _ptr(match),
                                                      query.numel(), ctypes.byref(n)))
        return n.value


    # ---- active-list keypoints ------------------------------------------
    def cloud_resolution(self, x, y, z):
        """Keypoints::computeCloudResolution (keypoints.h:401-428), host arrays."""
        x, y, z = map(_f32, (x, y, z))
        out = ctypes.c_double()
        self._check(self._lib.pfx_cloud_resolution(self.h, _ptr(x), _ptr(y), _ptr(z), len(x), ctypes.byref(out)))
        return out.value

    def cloud_resolution_dev(self, x, y, z):
        """Keypoints::computeCloudResolution on device arrays (the value comes back to the host,
        as the reference's return value)."""
        out = ctypes.c_double()
        self._check(self._lib.pfx_cloud_resolution_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(),
                                                       ctypes.byref(out)))
        return out.value

    def iss_keypoints(self, x, y, z, salient_radius, non_max_radius, min_neighbors=5, threshold21=0.975,
                      threshold32=0.975, return_third=False):
        """ISSKeypoint3D::compute (keypoints.h:177-189), host arrays: keypoint indices ascending
        (and the per-point third eigenvalue map)."""
        x, y, z = map(_f32, (x, y, z))
        n = len(x)
        idx = np.empty(max(n, 1), np.int32)
        third = np.empty(max(n, 1), np.float64) if return_third else None
        k = ctypes.c_int64()
        self._check(self._lib.pfx_iss_keypoints(self.h, _ptr(x), _ptr(y), _ptr(z), n, salient_radius, non_max_radius,
                                                min_neighbors, threshold21, threshold32, _ptr(idx), len(idx),
                                                ctypes.byref(k), _ptr(third)))
        out = idx[: k.value].copy()
        return (out, third[:n].copy()) if return_third else out

    def iss_keypoints_dev(self, x, y, z, salient_radius, non_max_radius, idx, min_neighbors=5, threshold21=0.975,
                          threshold32=0.975, third=None):
        """Device version: indices into `idx` (int32 tensor), returns their number."""
        k = ctypes.c_int64()
        self._check(self._lib.pfx_iss_keypoints_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), salient_radius,
                                                    non_max_radius, min_neighbors, threshold21, threshold32,
                                                    _ptr(idx), idx.numel(), ctypes.byref(k), _ptr(third)))
        return k.value

    def harris3d_keypoints(self, x, y, z, radius=0.01, threshold=1e-6, refine=True, non_max=True, details=False):
        """HarrisKeypoint3D + getKeypointsCloud (keypoints.h:150-162, 365-395), host arrays: the
        snapped cloud indices in corner order (details: and the per-point response and the
        refined corners)."""
        x, y, z = map(_f32, (x, y, z))
        n = len(x)
        cap = max(n, 1)
        idx = np.empty(cap, np.int32)
        resp = np.empty(cap, np.float32) if details else None
        corners = np.empty((cap, 3), np.float32) if details else None
        k, nc = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.pfx_harris3d_keypoints(self.h, _ptr(x), _ptr(y), _ptr(z), n, radius, threshold,
                                                     1 if non_max else 0, 1 if refine else 0, _ptr(idx), cap,
                                                     ctypes.byref(k), _ptr(resp), _ptr(corners), ctypes.byref(nc),
                                                     None))
        out = idx[: k.value].copy()
        return (out, resp[:n].copy(), corners[: nc.value].copy()) if details else out

    def harris3d_keypoints_dev(self, x, y, z, idx, radius=0.01, threshold=1e-6, refine=True, response=None,
                               corners=None):
        """Device version: snapped indices into `idx` (int32 tensor); returns (count, corners)."""
        k, nc = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.pfx_harris3d_keypoints_dev(self.h, _ptr(x), _ptr(y), _ptr(z), x.numel(), radius,
                                                         threshold, 1, 1 if refine else 0, _ptr(idx), idx.numel(),
                                                         ctypes.byref(k), _ptr(response), _ptr(corners),
                                                         ctypes.byref(nc), None))
        return k.value, nc.value

    def harris6d_keypoints(self, x, y, z, rgb, radius=0.01, threshold=1e-6, refine=True, non_max=True,
                           details=False):
        """HarrisKeypoint6D + getKeypointsCloud (keypoints.h:164-176, 365-395), host arrays (rgb:
        packed 0x00RRGGBB per point): the snapped cloud indices in corner order (details: and the
        per-point response, the refined corners and the normalised intensity gradients (n, 3))."""
        x, y, z = map(_f32, (x, y, z))
        rgb = np.ascontiguousarray(rgb, dtype=np.uint32)
        n = len(x)
        if len(rgb) != n:
            raise ValueError("harris6d: one rgb word per point")
        cap = max(n, 1)
        idx = np.empty(cap, np.int32)
        resp = np.empty(cap, np.float32) if details else None
        corners = np.empty((cap, 3), np.float32) if details else None
        grad = np.empty((cap, 3), np.float32) if details else None
        k, nc = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.pfx_harris6d_keypoints(self.h, _ptr(x), _ptr(y), _ptr(z), _ptr(rgb), n, radius,
                                                     threshold, 1 if non_max else 0, 1 if refine else 0, _ptr(idx),
                                                     cap, ctypes.byref(k), _ptr(resp), _ptr(corners), ctypes.byref(nc),
                                                     _ptr(grad), None))
        out = idx[: k.value].copy()
        return (out, resp[:n].copy(), corners[: nc.value].copy(), grad[:n].copy()) if details else out

    def harris6d_keypoints_dev(self, x, y, z, rgb, idx, radius=0.01, threshold=1e-6, refine=True, response=None,
                               corners=None, grad=None):
        """Device version (rgb: int32/uint32 tensor of packed colours): snapped indices into `idx`
        (int32 tensor); returns (count, corners)."""
        k, nc = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.pfx_harris6d_keypoints_dev(self.h, _ptr(x), _ptr(y), _ptr(z), _ptr(rgb), x.numel(),
                                                         radius, threshold, 1, 1 if refine else 0, _ptr(idx),
                                                         idx.numel(), ctypes.byref(k), _ptr(response), _ptr(corners),
                                                         ctypes.byref(nc), _ptr(grad), None))
        return k.value, nc.value

    # ---- RANSAC correspondence rejection -----------------------------------
    def ransac_rejector(self, src, tgt, query, match, threshold=0.015, max_iterations=1000):
        """Features::filterCorrespondences (features.h:282-297): (kept correspondence positions in
        input order, best 4x4 transformation).  src / tgt: (n, 3) keypoint clouds (host)."""
        src = np.ascontiguousarray(src, np.float32)
        tgt = np.ascontiguousarray(tgt, np.float32)
        sx, sy, sz = (np.ascontiguousarray(src[:, i]) for i in range(3))
        tx, ty, tz = (np.ascontiguousarray(tgt[:, i]) for i in range(3))
        query = np.ascontiguousarray(query, np.int32)
        match = np.ascontiguousarray(match, np.int32)
        n = len(query)
        keep = np.empty(max(n, 1), np.int32)
        T = np.empty(16, np.float32)
        nk = ctypes.c_int64()
        self._check(self._lib.pfx_ransac_rejector(self.h, _ptr(sx), _ptr(sy), _ptr(sz), len(sx), _ptr(tx), _ptr(ty),
                                                  _ptr(tz), len(tx), _ptr(query), _ptr(match), n, threshold,
                                                  max_iterations, _ptr(keep), ctypes.byref(nk), _ptr(T)))
        return keep[: nk.value].copy(), T.reshape(4, 4)


def batch_plan(n_scans, n_devices, rows_per_scan=None):
    """pfx_batch_plan (host only, no device): (device_of_scan, slot_of_scan, row_offset[n_scans + 1])
    of the batch's round-robin deal and scan-order gather layout."""
    lib = N.lib()
    n_scans = int(n_scans)
    if n_scans < 0:  # (checked here: np.zeros(n_scans + 1) would raise a numpy error first)
        raise N.PfxError(N.PFX_ERR_INVALID, f"pfx_batch_plan: n_scans = {n_scans} < 0")
    rows = None if rows_per_scan is None else np.ascontiguousarray(rows_per_scan, np.int64).ravel()
    if rows is not None and len(rows) != n_scans:  # the C side reads rows_per_scan[0..n_scans)
        raise N.PfxError(N.PFX_ERR_INVALID,
                         f"pfx_batch_plan: rows_per_scan has {len(rows)} entries for {n_scans} scans")
    dev = np.zeros(max(n_scans, 1), np.int32)
    slot = np.zeros(max(n_scans, 1), np.int32)
    off = np.zeros(n_scans + 1, np.int64)
    st = lib.pfx_batch_plan(int(n_scans), int(n_devices), None if rows is None else _ptr(rows), _ptr(dev), _ptr(slot),
                            _ptr(off))
    if st != 0:
        raise N.PfxError(st, "pfx_batch_plan")
    return dev[:n_scans], slot[:n_scans], off


class Batch:
    """pfx_batch: the multi-GPU scan batch of one process; scan s on devices[s % G],
    results gathered on devices[0] over RCCL and returned in scan order."""

    def __init__(self, devices=(0,)):
        self._lib = N.lib()
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = ctypes.c_void_p()
        st = self._lib.pfx_batch_create(devs.ctypes.data_as(ctypes.c_void_p), len(devs), ctypes.byref(h))
        if st != 0:
            raise N.PfxError(st, "pfx_batch_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._lib.pfx_batch_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def narf_fpfh(self, clouds, normal_radius=0.05, feature_radius=0.08, params=None, cam=None, cap_rows=1 << 20):
        """clouds: list of (x, y, z) host arrays.  Returns [(K_s x 33 descriptors, K_s cloud indices)]."""
        cl = [tuple(_f32(a) for a in c) for c in clouds]
        ns = len(cl)
        arr = lambda i: (ctypes.c_void_p * max(ns, 1))(*[c[i].ctypes.data for c in cl])  # noqa: E731
        xs, ys, zs = arr(0), arr(1), arr(2)
        n = np.array([len(c[0]) for c in cl], np.int64)
        desc = np.empty((cap_rows, 33), np.float32)
        idx = np.empty(cap_rows, np.int32)
        rows = np.zeros(max(ns, 1), np.int64)
        st = self._lib.pfx_batch_narf_fpfh(self.h, ns, xs, ys, zs, _ptr(n), ctypes.byref(cam or camera()),
                                           ctypes.byref(params or narf_params(support_size=0.2)),
                                           float(normal_radius), float(feature_radius), _ptr(desc), _ptr(idx),
                                           cap_rows, _ptr(rows))
        if st != 0:
            raise N.PfxError(st, self._lib.pfx_batch_last_error(self.h).decode())
        out, o = [], 0
        for k in rows[:ns]:
            out.append((desc[o:o + k].copy(), idx[o:o + k].copy()))
            o += int(k)
        return out
