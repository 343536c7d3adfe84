"""Seeded synthetic clouds of BASELINE.json's configs.

* ``synth_room(N, seed)`` -- pinhole back-projection of uniform continuous pixels
  (u, v) in [0,640) x [0,480) (f = 525, c = (320, 240), the reference's NARF camera,
  keypoints.h:203-207) onto a piecewise room (floor, back wall, side wall, 3 boxes, 1 sphere)
  spanning z in [1, 4]*s, with Gaussian noise along the ray (sigma = 1.5 mm) and
  s = 0.58 sqrt(N / 1e5) (SURVEY's sqrt(N/1e5) times a calibration factor for this scene), so
  the surface density -- and the mean radius-0.05 neighbour count -- does not change with N
  (k(0.05) ~ 230 as on data/indoor).
* ``synth_seabed(N, seed)`` -- a camera looking down at a height field
  z = D + 0.08 fbm(x, y) (5 octaves), D chosen for the data/underwater density
  (k(0.05) ~ 400, k(0.08) ~ 930).

Points are float32 SoA in metres, VIEWPOINT identity, every point in front of the camera and
inside the 640x480 image, rgb = random packed 0x00RRGGBB (unused by the path).
"""
from __future__ import annotations

import numpy as np

F, CX, CY, W, H = 525.0, 320.0, 240.0, 640, 480


def _rays(rng, n):
    u = rng.uniform(0.0, W, n)
    v = rng.uniform(0.0, H, n)
    return (u - CX) / F, (v - CY) / F


def _plane_t(d, axis, value):
    with np.errstate(divide="ignore", invalid="ignore"):
        t = value / d[axis]
    return np.where(t > 1e-6, t, np.inf)


def _box_t(d, lo, hi):
    """Slab-method entry distance of rays from the origin into an axis-aligned box."""
    with np.errstate(divide="ignore", invalid="ignore"):
        t0 = np.full(d[0].shape, -np.inf)
        t1 = np.full(d[0].shape, np.inf)
        for a in range(3):
            inv = 1.0 / d[a]
            ta = lo[a] * inv
            tb = hi[a] * inv
            t0 = np.maximum(t0, np.minimum(ta, tb))
            t1 = np.minimum(t1, np.maximum(ta, tb))
    hit = (t1 >= t0) & (t0 > 1e-6)
    return np.where(hit, t0, np.inf)


def _sphere_t(d, c, r):
    a = d[0] ** 2 + d[1] ** 2 + d[2] ** 2
    b = -2.0 * (d[0] * c[0] + d[1] * c[1] + d[2] * c[2])
    cc = c[0] ** 2 + c[1] ** 2 + c[2] ** 2 - r * r
    disc = b * b - 4 * a * cc
    with np.errstate(invalid="ignore"):
        t = (-b - np.sqrt(disc)) / (2 * a)
    return np.where((disc >= 0) & (t > 1e-6), t, np.inf)


def _finish(rng, d, t, n, sigma=0.0015):
    norm = np.sqrt(d[0] ** 2 + d[1] ** 2 + d[2] ** 2)
    t = t + rng.normal(0.0, sigma, n) / norm  # noise along the ray, sigma in metres
    x = (d[0] * t).astype(np.float32)
    y = (d[1] * t).astype(np.float32)
    z = (d[2] * t).astype(np.float32)
    rgb = rng.integers(0, 1 << 24, n, dtype=np.uint32)
    return x, y, z, rgb


ROOM_SCALE = 0.58  # calibrated: mean radius-0.05 neighbour count ~ 230 (data/indoor: 233)


def synth_room(n: int, seed: int = 1, scale: float = ROOM_SCALE):
    rng = np.random.default_rng(seed)
    s = scale * float(np.sqrt(n / 1e5))
    dx, dy = _rays(rng, n)
    d = (dx, dy, np.ones(n))
    ts = [
        _plane_t(d, 2, 4.0 * s),          # back wall
        _plane_t(d, 1, 0.75 * s),         # floor (image y points down)
        _plane_t(d, 0, -1.45 * s),        # left side wall
        _box_t(d, np.array([-0.85, 0.20, 2.0]) * s, np.array([-0.20, 0.75, 2.6]) * s),
        _box_t(d, np.array([0.30, 0.05, 2.8]) * s, np.array([1.05, 0.75, 3.4]) * s),
        _box_t(d, np.array([-0.25, 0.40, 1.0]) * s, np.array([0.20, 0.75, 1.35]) * s),
        _sphere_t(d, np.array([0.85, -0.10, 2.1]) * s, 0.33 * s),
    ]
    t = np.minimum.reduce(ts)
    t = np.where(np.isfinite(t), t, 4.0 * s)
    return _finish(rng, d, t, n)


def _fbm(x, y, seed, octaves=5):
    rng = np.random.default_rng(seed + 7919)
    v = np.zeros_like(x)
    amp, freq = 0.5, 1.6
    for _ in range(octaves):
        kx, ky = rng.normal(size=2)
        ph = rng.uniform(0, 2 * np.pi, 2)
        v += amp * np.sin(freq * (kx * x + ky * y) + ph[0]) * np.cos(freq * (ky * x - kx * y) + ph[1])
        amp *= 0.5
        freq *= 2.03
    return v


def synth_seabed(n: int, seed: int = 3, depth: float | None = None):
    rng = np.random.default_rng(seed)
    # k(0.05) ~ 400 at n = 1M: pixel footprint ~ 8 mm  ->  D ~ 4.2 m; scale with sqrt(n)
    D = depth if depth is not None else 4.2 * float(np.sqrt(n / 1e6))
    dx, dy = _rays(rng, n)
    t = np.full(n, D)
    for _ in range(6):  # fixed point: t = D + 0.08 fbm(t dx, t dy)
        t = D + 0.08 * _fbm(t * dx, t * dy, seed)
    d = (dx, dy, np.ones(n))
    return _finish(rng, d, t, n)


def texture_rgb(x, y, z, seed: int = 0):
    """Packed 0x00RRGGBB colours of a smooth procedural texture (stripes and blobs at 2-10 cm
    scales) over the scene: colour gradients for HarrisKeypoint6D (the generators' own rgb is
    uniform noise, which the xyz-only path never reads)."""
    rng = np.random.default_rng(seed + 104729)
    x, y, z = (np.asarray(a, np.float64) for a in (x, y, z))
    ch = []
    for _ in range(3):
        k = rng.normal(size=(3, 3)) * np.array([[60.0], [90.0], [140.0]])
        ph = rng.uniform(0, 2 * np.pi, 3)
        v = 0.0
        for j in range(3):
            v = v + np.sin(k[j, 0] * x + k[j, 1] * y + k[j, 2] * z + ph[j]) / (j + 1)
        ch.append(np.clip(128.0 + 70.0 * v, 0, 255).astype(np.uint32))
    return (ch[0] << 16) | (ch[1] << 8) | ch[2]


def config(name: str):
    """The BASELINE.json configs as (x, y, z) generators."""
    if name == "cfg2_room100k":
        return synth_room(100_000, 1)
    if name == "cfg3_room1m":
        return synth_room(1_000_000, 2)
    if name == "cfg4_seabed1m":
        return synth_seabed(1_000_000, 3)
    raise KeyError(name)
