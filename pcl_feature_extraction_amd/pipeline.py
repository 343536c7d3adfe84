"""The reference's NARF + FPFH descriptor path as one device-resident pass.

Mirrors, for one scan, what src/evaluation.cpp does for the (Narf, FPFH) pair:
  Keypoints("Narf").compute(cloud, kps)        keypoints.h:199-231
      RangeImagePlanar 640x480 -> NarfKeypoint(support 0.2) -> pixel indices
      kps = cloud->points[pixel_index]          keypoints.h:227-229 (index quirk, guarded)
  Features<FPFHSignature33>(FPFHEstimation, 0.08, 0.05).compute(cloud, kps, desc)
      Tools::estimateNormals(cloud, r = 0.05)   features.h:187, tools.h:22-32
      FPFH(surface = cloud, input = kps, r = 0.08)   features.h:188-195
All arrays stay in HBM (torch tensors as device memory); the C-ABI calls are stream-ordered on
the ctx stream.  Nothing here computes on the CPU except NARF's greedy selection inside libpfx.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .api import Context, camera, narf_params


@dataclasses.dataclass
class ScanBuffers:
    x: object
    y: object
    z: object
    nx: object
    ny: object
    nz: object
    curv: object
    kx: object
    ky: object
    kz: object
    desc: object


def alloc(torch, n: int, device, max_keypoints: int = 1 << 16) -> ScanBuffers:
    f = dict(dtype=torch.float32, device=device)
    e = lambda m: torch.empty(m, **f)  # noqa: E731
    return ScanBuffers(e(n), e(n), e(n), e(n), e(n), e(n), e(n), e(max_keypoints), e(max_keypoints),
                       e(max_keypoints), torch.empty((max_keypoints, 33), **f))


def narf_fpfh(ctx: Context, b: ScanBuffers, normal_radius: float = 0.05, feat_radius: float = 0.08,
              params=None, cam=None):
    """Returns (keypoint pixel indices (np.int32), number of descriptor rows K)."""
    kp = ctx.narf_keypoints_dev(b.x, b.y, b.z, params or narf_params(support_size=0.2), cam or camera())
    k = ctx.gather_points_dev(b.x, b.y, b.z, kp, b.kx, b.ky, b.kz)
    ctx.normals_dev(b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)
    if k > 0:
        ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius, b.desc[:k])
    return kp, k


class OverlappedNarfFpfh:
    """narf_fpfh with the two independent halves of the pass overlapped on the device: NARF (+ the
    keypoint gather) on the main context/stream, normal estimation -- which needs only the cloud --
    on a second context/stream driven from a worker thread (the C-ABI calls release the GIL), then
    FPFH on the main stream after an event wait for the normals.  Same results as narf_fpfh.

    (Measured alternatives, not used: normals of the FPFH support set first -- a support mask +
    two masked pfx_normals_chains_dev passes -- so FPFH overlaps the other normals.  The exact
    support (pfx_fpfh_support_mask_dev) costs ~1 ms to mark: 11.0 vs 9.5 ms (round 1); the 2r
    ball (pfx_fpfh_support_ball_dev, 60 us) still holds most of the chain work, and the second
    pass's long-list kernel shares a hardware queue with FPFH: 7.44 vs 7.02 ms (round 2).)"""

    def __init__(self, torch, ctx_main: Context, ctx_side: Context, device, main_stream=None):
        from concurrent.futures import ThreadPoolExecutor
        self.torch = torch
        self.ctx, self.ctx_side = ctx_main, ctx_side
        self.s_main = main_stream if main_stream is not None else torch.cuda.current_stream(device)
        # the normal estimation is the step's critical path: its stream gets the higher priority,
        # so its short dependent launches (grid build, list set-up) are dispatched ahead of NARF's
        # workgroups (A/B: 166.6 -> 167.8 Mpoints/s)
        self.s_side = torch.cuda.Stream(device, priority=-1)
        ctx_main.set_stream(self.s_main.cuda_stream)
        ctx_side.set_stream(self.s_side.cuda_stream)
        ctx_main.set_shared(True)  # NARF shares the device with the critical normal estimation
        self.pool = ThreadPoolExecutor(max_workers=1)
        # opt-in: the MFMA-covariance normals (pfx_normals_fast_dev), not parity-exact
        self.fast_normals = False
        # FPFH's support first: normals of the points FPFH reads (pfx_fpfh_support_ball_dev), then
        # FPFH on the main stream while the side stream estimates the rest (same results)
        # (1: subset lists + chains, 2: every list, then the chains by workgroup partition)
        # (schedule attributes: every value is pinned by a -m gpu parity test against the default,
        # tests/test_gpu_pipeline.py)
        self.support_first = 0
        # "support": with support_first = 1, estimate only the support's normals -- the step's
        # outputs (keypoints, descriptors) are unchanged, as the normals are an intermediate of
        # Features::compute (features.h:185-187); the other normal outputs are left unwritten
        self.normals_scope = "all"
        # the normal estimation's validation off the critical path (pfx_normals_launch_dev /
        # pfx_normals_finish_dev, FPFH queued in between; A/B 173.8 vs 172.1 Mpoints/s, 3 runs each;
        # False: pfx_normals_dev, whose check precedes the chains)
        self.split_check = True
        # split form: the estimation's ~50 launches issued by the calling thread before NARF's (no
        # host round trip in them), the worker only waits for the check.  Two threads launching at
        # once contend inside the HIP runtime (~60 us per launch in the API trace instead of ~7),
        # which stretched the grid build at the head of the critical path.
        self.launch_first = True
        # with launch_first: FPFH's surface grid (it needs only the cloud) queued before NARF, so
        # after NARF's host selection only the keypoint gather and the S marking remain before SPFH
        # (1: after the estimation's launch; 2: before it, with the estimation's list kernels gated
        # on it -- pfx_normals_gate_dev -- so it never queues behind them; 0: after NARF)
        self.prep_first = 2
        # with prep_first == 2: the estimation's grid queued on the side stream before FPFH's
        # surface grid (pfx_normals_grid_launch_dev), the gated list kernels the only part that
        # waits for FPFH's.  Measured slower (r05 A/B, 3 runs each: 198.4 vs 204.5 Mpoints/s --
        # the normal stage gains 0.08 ms, the step loses 0.15 ms to NARF and FPFH's grid queued
        # behind it), so off; pinned by tests/test_gpu_pipeline.py
        self.grid_first = False
        # shot(): the SHOT surface grid queued before the normal estimation, whose list kernels then
        # wait for it (pfx_normals_gate_dev), instead of after NARF (where its radix sort runs beside
        # the persistent list kernels, ~0.85 ms instead of ~0.03).  Measured (r05, 2 runs each):
        # 197.0 / 198.2 vs 198.2 / 199.5 Mpoints/s, so off; pinned by tests/test_gpu_pipeline.py
        self.shot_prep_first = False
        self._support = None

    def __call__(self, b: ScanBuffers, normal_radius: float = 0.05, feat_radius: float = 0.08, params=None,
                 cam=None):
        self.s_side.wait_stream(self.s_main)  # the scan was written on the main stream
        if self.support_first and not self.fast_normals:
            return self._support_first(b, normal_radius, feat_radius, params, cam)
        ev = self.torch.cuda.Event()
        split = self.split_check and not self.fast_normals
        if split and self.launch_first:
            if self.prep_first == 2:
                if self.grid_first:
                    self.ctx_side.normals_grid_launch_dev(b.x, b.y, b.z, normal_radius)
                self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
                gate = self.torch.cuda.Event()
                gate.record(self.s_main)
                self.ctx_side.normals_gate_dev(gate)
            self.ctx_side.normals_launch_dev(b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)
            ev.record(self.s_side)
            launched = None
            fut = self.pool.submit(self.ctx_side.normals_finish_dev)
            if self.prep_first == 1:
                self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
        elif split:
            # the estimation queued with no host round trip, FPFH queued right behind it, and its
            # validation (pfx_normals_finish_dev) on the worker while FPFH is being queued
            import threading
            launched = threading.Event()

            def est(*a):
                try:
                    self.ctx_side.normals_launch_dev(*a)
                    ev.record(self.s_side)
                finally:
                    launched.set()
                return self.ctx_side.normals_finish_dev()
        else:
            launched = None
            est = self.ctx_side.normals_fast_dev if self.fast_normals else self.ctx_side.normals_dev
        if not (split and self.launch_first):
            fut = self.pool.submit(est, b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)
        rerun = False
        try:
            kp = self.ctx.narf_keypoints_dev(b.x, b.y, b.z, params or narf_params(support_size=0.2),
                                             cam or camera())
            k = self.ctx.gather_points_dev(b.x, b.y, b.z, kp, b.kx, b.ky, b.kz)
            # the FPFH surface grid (normals-free) after NARF: the step's first milliseconds
            # belong to the normal-estimation grid and NARF, the critical and the longer path
            if not (split and self.launch_first and self.prep_first):  # (already queued)
                self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
            if k > 0:  # FPFH's SPFH point set, also normals-free
                self.ctx.fpfh_prepare_queries_dev(b.x, b.y, b.z, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius)
            if split:
                if launched is not None:
                    launched.wait()
                self.s_main.wait_event(ev)
                if k > 0:
                    self.ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius,
                                      b.desc[:k])
        finally:
            rerun = fut.result()
        if split:
            if rerun:  # the estimation was rerun exactly: FPFH again, behind it
                self.s_main.wait_stream(self.s_side)
                if k > 0:
                    self.ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius,
                                      b.desc[:k])
            return kp, k
        ev.record(self.s_side)
        self.s_main.wait_event(ev)
        if k > 0:
            self.ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius,
                              b.desc[:k])
        return kp, k

    def _support_first(self, b: ScanBuffers, normal_radius, feat_radius, params, cam):
        """The normal estimation in two subsets (pfx_normals_subset_dev): the FPFH support -- every
        point within 2 feat_radius of a keypoint, a superset of the normals FPFHEstimation reads --
        as soon as NARF has found the keypoints, then the rest, concurrently with FPFH.  The side
        stream builds the grid while NARF runs; both subsets finish inside the call."""
        import threading
        torch = self.torch
        n = b.x.numel()
        if self._support is None or self._support.numel() < n:
            self._support = torch.empty(n, dtype=torch.uint8, device=b.x.device)
        sup = self._support[:n]
        mask_ready, sup_done = threading.Event(), threading.Event()
        ev_mask, ev_sup = torch.cuda.Event(), torch.cuda.Event()
        failed = []

        cs = self.ctx_side
        split = self.support_first == 2

        def normals():
            try:
                if split:
                    cs.normals_lists_dev(b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)
                else:
                    cs.normals_prepare_dev(b.x, b.y, b.z, normal_radius)
                mask_ready.wait()
                if failed:
                    return
                self.s_side.wait_event(ev_mask)
                if split:
                    cs.normals_chains_dev(cs, b.nx, b.ny, b.nz, b.curv, mask=sup, want=3)
                else:
                    cs.normals_subset_dev(b.x, b.y, b.z, normal_radius, sup, 1, b.nx, b.ny, b.nz, b.curv)
                ev_sup.record(self.s_side)
            finally:
                sup_done.set()
            if split:
                cs.normals_chains_dev(cs, b.nx, b.ny, b.nz, b.curv, mask=sup, want=2)
            elif self.normals_scope != "support":
                cs.normals_subset_dev(b.x, b.y, b.z, normal_radius, sup, 0, b.nx, b.ny, b.nz, b.curv)

        fut = self.pool.submit(normals)
        k = 0
        try:
            try:
                kp = self.ctx.narf_keypoints_dev(b.x, b.y, b.z, params or narf_params(support_size=0.2),
                                                 cam or camera())
                k = self.ctx.gather_points_dev(b.x, b.y, b.z, kp, b.kx, b.ky, b.kz)
                self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
                if k > 0:
                    self.ctx.fpfh_prepare_queries_dev(b.x, b.y, b.z, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius)
                    self.ctx.fpfh_support_ball_dev(b.x, b.y, b.z, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius, sup)
                else:
                    sup.zero_()
                ev_mask.record(self.s_main)
            except BaseException:
                failed.append(True)
                raise
            finally:
                mask_ready.set()
            sup_done.wait()
            self.s_main.wait_event(ev_sup)
            if k > 0:
                self.ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius,
                                  b.desc[:k])
        finally:
            fut.result()
        self.s_main.wait_stream(self.s_side)  # every normal belongs to the step
        return kp, k

    def shot(self, b: ScanBuffers, s, sample, normal_radius: float = 0.05, feat_radius: float = 0.08,
             params=None, cam=None):
        """narf_shot with the same overlap: the normal estimation on the side stream while NARF,
        the keypoint gather, the sample's coordinates and the SHOT surface grid
        (pfx_fpfh_prepare_dev's, which shot_dev takes over) run on the main stream; SHOT after an
        event on the normals.  Same results as narf_shot; returns the number of rows."""
        import threading
        torch = self.torch
        self.s_side.wait_stream(self.s_main)
        ev = torch.cuda.Event()
        launched = threading.Event()

        def est(*a):  # (as __call__'s split check: SHOT queued behind the launched estimation)
            try:
                self.ctx_side.normals_launch_dev(*a)
                ev.record(self.s_side)
            finally:
                launched.set()
            return self.ctx_side.normals_finish_dev()

        if self.shot_prep_first:
            self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
            gate = torch.cuda.Event()
            gate.record(self.s_main)
            self.ctx_side.normals_gate_dev(gate)
        fut = self.pool.submit(est, b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)

        def run_shot():
            self.ctx.shot_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, s.qx[:rows], s.qy[:rows], s.qz[:rows], feat_radius,
                              s.desc[:rows], s.rf[:rows])

        rerun = False
        try:
            kp = self.ctx.narf_keypoints_dev(b.x, b.y, b.z, params or narf_params(support_size=0.2),
                                             cam or camera())
            k = self.ctx.gather_points_dev(b.x, b.y, b.z, kp, s.qx, s.qy, s.qz)
            m = sample.numel()
            with torch.cuda.stream(self.s_main):
                torch.index_select(b.x, 0, sample, out=s.qx[k:k + m])
                torch.index_select(b.y, 0, sample, out=s.qy[k:k + m])
                torch.index_select(b.z, 0, sample, out=s.qz[k:k + m])
            if not self.shot_prep_first:
                self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
            rows = k + m
            launched.wait()
            self.s_main.wait_event(ev)
            run_shot()
        finally:
            rerun = fut.result()
        if rerun:  # the estimation was rerun exactly: SHOT again, behind it
            self.s_main.wait_stream(self.s_side)
            run_shot()
        return rows

    def check(self):
        """Once per batch, outside any timed region: synchronises both contexts so errors the
        stream-ordered calls defer (an FPFH neighbourhood beyond capacity) are raised."""
        self.ctx_side.synchronize()
        self.ctx.synchronize()

    def close(self):
        self.pool.shutdown()


class BatchNarfFpfh:
    """The (Narf, FPFH) pass over a batch of device-resident scans on one GPU -- the per-scan loop
    of evaluation.cpp:272-852 for the scans a rank owns (configs[4]) -- software-pipelined over two
    streams: a worker thread issues every scan's normal estimation back to back on the side stream
    (the step's critical path), while the calling thread issues scan i's NARF + keypoint gather +
    FPFH surface/S preparation on the main stream and then scan i's FPFH behind an event on scan
    i's normals.  So scan i's FPFH and scan i+1's NARF overlap scan i+1's normal estimation.
    Results are those of narf_fpfh per scan (same kernels, same contexts per role)."""

    def __init__(self, torch, ctx_main: Context, ctx_side: Context, device, main_stream=None, side_stream=None):
        self.torch = torch
        self.ctx, self.ctx_side = ctx_main, ctx_side
        self.s_main = main_stream if main_stream is not None else torch.cuda.current_stream(device)
        # side_stream: share an OverlappedNarfFpfh's stream when both drive the same contexts
        self.s_side = side_stream if side_stream is not None else torch.cuda.Stream(device, priority=-1)
        ctx_main.set_stream(self.s_main.cuda_stream)
        ctx_side.set_stream(self.s_side.cuda_stream)
        ctx_main.set_shared(True)
        from concurrent.futures import ThreadPoolExecutor
        self.pool = ThreadPoolExecutor(max_workers=1)

    def __call__(self, scans, normal_radius: float = 0.05, feat_radius: float = 0.08, params=None, cam=None):
        """scans: list of ScanBuffers (coordinates written on the main stream before this call).
        Returns [(kp pixel indices, K)] in scan order; descriptors in each scan's b.desc[:K]."""
        import threading
        torch = self.torch
        self.s_side.wait_stream(self.s_main)
        done = [threading.Event() for _ in scans]
        evs = [torch.cuda.Event() for _ in scans]

        failed = []

        def normals_all():
            try:
                for i, b in enumerate(scans):
                    self.ctx_side.normals_dev(b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)
                    evs[i].record(self.s_side)
                    done[i].set()
            except BaseException as e:
                failed.append(e)
                for d in done:  # release the issuing thread wherever it waits
                    d.set()
                raise

        fut = self.pool.submit(normals_all)
        out = []
        try:
            for i, b in enumerate(scans):
                kp = self.ctx.narf_keypoints_dev(b.x, b.y, b.z, params or narf_params(support_size=0.2),
                                                 cam or camera())
                k = self.ctx.gather_points_dev(b.x, b.y, b.z, kp, b.kx, b.ky, b.kz)
                self.ctx.fpfh_prepare_dev(b.x, b.y, b.z, feat_radius)
                if k > 0:
                    self.ctx.fpfh_prepare_queries_dev(b.x, b.y, b.z, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius)
                done[i].wait()
                if failed:
                    raise failed[0]
                self.s_main.wait_event(evs[i])
                if k > 0:
                    self.ctx.fpfh_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, b.kx[:k], b.ky[:k], b.kz[:k], feat_radius,
                                      b.desc[:k])
                out.append((kp, k))
        finally:
            fut.result()
        return out

    def check(self):
        """Raises deferred errors of the stream-ordered calls (see OverlappedNarfFpfh.check)."""
        self.ctx_side.synchronize()
        self.ctx.synchronize()

    def close(self):
        self.pool.shutdown()


def keypoint_rows(kp: np.ndarray, n: int) -> np.ndarray:
    """Cloud indices the descriptors belong to (keypoints.h:229 uses pixel index as cloud index)."""
    kp = np.asarray(kp)
    return kp[(kp >= 0) & (kp < n)]


class DeviceRows:
    """keypoint_rows on the device, staged through a ring of pinned host blocks so the copy is a
    real async DMA.  (A pageable-memory copy blocks the host until its stream reaches it -- i.e.
    until the scan's FPFH has finished -- so the next scan's launches were queued only after the
    device had drained: ~0.25 ms of idle device per scan.)  A slot is reused `slots` calls later,
    after its copy's event; the device block returned stays valid until then."""

    def __init__(self, torch, device, slots: int = 2, cap: int = 1 << 16):
        self.torch, self.device = torch, device
        self.h = [torch.empty(cap, dtype=torch.int32, pin_memory=True) for _ in range(slots)]
        self.d = [torch.empty(cap, dtype=torch.int32, device=device) for _ in range(slots)]
        self.ev = [None] * slots
        self.i = 0

    def __call__(self, kp: np.ndarray, n: int):
        rows = keypoint_rows(kp, n).astype(np.int32)
        s = self.i
        self.i = (s + 1) % len(self.h)
        if self.ev[s] is not None:
            self.ev[s].synchronize()
        k = len(rows)
        if k > self.h[s].numel():
            self.h[s] = self.torch.empty(k, dtype=self.torch.int32, pin_memory=True)
            self.d[s] = self.torch.empty(k, dtype=self.torch.int32, device=self.device)
        self.h[s][:k].numpy()[:] = rows
        out = self.d[s][:k]
        out.copy_(self.h[s][:k], non_blocking=True)
        ev = self.torch.cuda.Event()
        ev.record()
        self.ev[s] = ev
        return out


@dataclasses.dataclass
class ShotBuffers:
    qx: object
    qy: object
    qz: object
    desc: object
    rf: object


def alloc_shot(torch, nq: int, device) -> ShotBuffers:
    f = dict(dtype=torch.float32, device=device)
    return ShotBuffers(torch.empty(nq, **f), torch.empty(nq, **f), torch.empty(nq, **f),
                       torch.empty((nq, 352), **f), torch.empty((nq, 9), **f))


def narf_shot(ctx: Context, b: ScanBuffers, s: ShotBuffers, sample, normal_radius: float = 0.05,
              feat_radius: float = 0.08, params=None, cam=None):
    """configs[3]: normals, then SHOT-352 at the NARF keypoints followed by a
    fixed sample of cloud indices (`sample`: int64 CUDA tensor).  Returns the number of rows."""
    import torch
    kp = ctx.narf_keypoints_dev(b.x, b.y, b.z, params or narf_params(support_size=0.2), cam or camera())
    k = ctx.gather_points_dev(b.x, b.y, b.z, kp, s.qx, s.qy, s.qz)
    m = sample.numel()
    torch.index_select(b.x, 0, sample, out=s.qx[k:k + m])
    torch.index_select(b.y, 0, sample, out=s.qy[k:k + m])
    torch.index_select(b.z, 0, sample, out=s.qz[k:k + m])
    ctx.normals_dev(b.x, b.y, b.z, normal_radius, b.nx, b.ny, b.nz, b.curv)
    rows = k + m
    ctx.shot_dev(b.x, b.y, b.z, b.nx, b.ny, b.nz, s.qx[:rows], s.qy[:rows], s.qz[:rows], feat_radius,
                 s.desc[:rows], s.rf[:rows])
    return rows


def keypoints_iss(ctx: Context, x, y, z, idx, third=None) -> int:
    """Keypoints("ISS").compute (keypoints.h:177-189): resolution = computeCloudResolution
    (keypoints.h:401-428), then ISSKeypoint3D with salient radius 6 res, non-max radius 4 res,
    min neighbours 5, thresholds 0.975 / 0.975.  Keypoint cloud indices (ascending) into `idx`;
    returns their number (0 for a cloud without two finite points: the reference's ISS then
    rejects the zero radius in initCompute and leaves the output empty)."""
    res = ctx.cloud_resolution_dev(x, y, z)
    if res <= 0.0:
        return 0
    return ctx.iss_keypoints_dev(x, y, z, 6 * res, 4 * res, idx, min_neighbors=5, threshold21=0.975,
                                 threshold32=0.975, third=third)


def keypoints_harris3d(ctx: Context, x, y, z, idx) -> int:
    """Keypoints("Harris3D").compute (keypoints.h:150-162): HarrisKeypoint3D<PointXYZRGB,
    PointXYZI> with non-maximum suppression, threshold 1e-6, radius 0.01 (the constructor's
    default) and corner refinement, then getKeypointsCloud (keypoints.h:365-395): the snapped
    cloud indices into `idx`; returns their number."""
    k, _ = ctx.harris3d_keypoints_dev(x, y, z, idx, radius=0.01, threshold=1e-6, refine=True)
    return k


def keypoints_harris6d(ctx: Context, x, y, z, rgb, idx) -> int:
    """Keypoints("Harris6D").compute (keypoints.h:164-176): HarrisKeypoint6D<PointXYZRGB,
    PointXYZI> with non-maximum suppression, threshold 1e-6, radius 0.01 (the constructor's
    default) and corner refinement, then getKeypointsCloud (keypoints.h:365-395); rgb: the
    cloud's packed colours (int32 tensor).  Snapped cloud indices into `idx`; returns their number."""
    k, _ = ctx.harris6d_keypoints_dev(x, y, z, rgb, idx, radius=0.01, threshold=1e-6, refine=True)
    return k
