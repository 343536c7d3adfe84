"""GPU parity of the NARF keypoint branch (keypoints.h:199-231) against the CPU restatement.

Bar: range image, border traits, surface-change scores, the interest image and the keypoint
pixel indices are all bit-exact (the index list is what NarfKeypoint::compute returns).
Parity vs real PCL is unpinned (oracle/or_narf.cpp header).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from parity import bits, bits_equal
from pcl_feature_extraction_amd.pcd import read_pcd

pytestmark = pytest.mark.gpu

CLOUDS = ["indoor_source", "indoor_target", "underwater_source", "underwater_target"]


def _cloud(name):
    c = read_pcd(os.path.join(os.path.dirname(__file__), "golden", "clouds", name + ".pcd"))
    return c.x, c.y, c.z


def _same(a, b):
    """Raw 32-bit patterns, NaN pixels included (a NaN with another payload is a mismatch)."""
    return bits_equal(np.asarray(a, np.float32).ravel(), np.asarray(b, np.float32).ravel())


@pytest.mark.parametrize("name", CLOUDS)
def test_range_image_bit_exact(ctx, name):
    x, y, z = _cloud(name)
    g = ctx.range_image_planar(x, y, z)
    o = O.range_image_planar(x, y, z)
    assert _same(g, o)


@pytest.mark.parametrize("name", CLOUDS)
def test_narf_keypoints_bit_exact(ctx, name):
    from pcl_feature_extraction_amd import narf_params
    x, y, z = _cloud(name)
    okp, dbg = O.narf_keypoints(x, y, z, debug=True)
    # dense interest image (calculate_sparse_interest_image = false): every pixel bit-exact
    kp_dense = ctx.narf_keypoints(x, y, z, params=narf_params(calculate_sparse_interest_image=0))
    traits = ctx.narf_debug_image("border_traits")
    scs = ctx.narf_debug_image("surface_change")
    interest = ctx.narf_debug_image("interest")
    assert np.array_equal(traits, dbg["border_traits"]), "border traits differ"
    assert _same(scs, dbg["surface_change"]), "surface change scores differ"
    assert _same(interest, dbg["interest"]), "interest image differs"
    assert np.array_equal(kp_dense, okp)
    # PCL's default sparse mode: same keypoints; the interest image is exact wherever it can
    # reach min_interest_value and 0 (skipped) or exact elsewhere
    kp = ctx.narf_keypoints(x, y, z)
    sparse = np.asarray(ctx.narf_debug_image("interest"), np.float32).ravel()
    dense = np.asarray(dbg["interest"], np.float32).ravel()
    hi = dense >= 0.45
    assert np.array_equal(sparse[hi].view(np.uint32), dense[hi].view(np.uint32))
    assert np.all((sparse[~hi] == 0) | (bits(sparse[~hi]) == bits(dense[~hi])))
    assert np.array_equal(kp, okp)
    assert len(kp) > 0
    assert np.all(np.diff(kp) > 0)  # ascending pixel indices
    # the boundary reports which interest formula ran: the complete one, in both modes
    # (PCL's own sparse heuristics are not reproduced; pfx.h pfx_narf_params)
    assert ctx.stat("narf_interest_formula") == 0


def test_narf_empty_cloud(ctx):
    e = np.zeros(0, np.float32)
    assert len(ctx.narf_keypoints(e, e, e)) == 0


def test_narf_points_behind_camera_ignored(ctx):
    x, y, z = _cloud("underwater_source")
    # mirror half the cloud behind the sensor: it must not change the image
    xb = np.concatenate([x, x[:5000]])
    yb = np.concatenate([y, y[:5000]])
    zb = np.concatenate([z, -z[:5000]])
    assert _same(ctx.range_image_planar(xb, yb, zb), O.range_image_planar(x, y, z))
    assert np.array_equal(ctx.narf_keypoints(xb, yb, zb), O.narf_keypoints(x, y, z))


def test_narf_every_region_grow_path(ctx):
    """Near-sensor points give region-grow windows beyond the flood-fill masks (> 128 px: queue
    grow in a windowed LDS bitmap) and beyond that bitmap (whole-image grow); the dense interest
    image must stay bit-exact on all three paths."""
    from pcl_feature_extraction_amd import narf_params
    from pcl_feature_extraction_amd.synth import synth_room
    x, y, z, _ = synth_room(40_000, 11)
    rng = np.random.default_rng(12)
    # a small box 0.16-0.5 m in front of the sensor: corners and edges (high surface change)
    u = rng.uniform(-0.03, 0.03, (3000, 2))
    near = np.c_[u, rng.choice([0.16, 0.5], 3000)].astype(np.float32)
    side = np.c_[np.full(1500, 0.03), rng.uniform(-0.03, 0.03, 1500), rng.uniform(0.16, 0.5, 1500)]
    pts = np.concatenate([np.c_[x, y, z], near, side.astype(np.float32)]).astype(np.float32)
    x, y, z = pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()
    dense = narf_params(calculate_sparse_interest_image=0)
    kp = ctx.narf_keypoints(x, y, z, params=dense)
    assert ctx.stat("narf_interest_queue_grown") > 0
    assert ctx.stat("narf_interest_fullimage") > 0
    okp, dbg = O.narf_keypoints(x, y, z, debug=True)
    assert _same(ctx.narf_debug_image("interest"), dbg["interest"])
    assert np.array_equal(kp, okp)
