"""GPU path against the committed oracle fixtures (tests/golden/oracle_small.npz): bit-exact."""
import os

import numpy as np
import pytest

from parity import bits_equal

pytestmark = pytest.mark.gpu
F = os.path.join(os.path.dirname(__file__), "golden", "oracle_small.npz")


def _eq(a, b):
    return bits_equal(a, b)  # raw bits, NaN rows included


def test_gpu_matches_golden_fixtures(ctx):
    f = np.load(F, allow_pickle=False)
    x, y, z, q = f["x"], f["y"], f["z"], f["queries"]
    n = np.stack(ctx.normals(x, y, z, 0.05))
    assert _eq(n, f["normals"])
    d = ctx.fpfh(x, y, z, n[0], n[1], n[2], x[q], y[q], z[q], 0.08)
    assert _eq(d, f["fpfh"])
    kp = ctx.narf_keypoints(f["narf_x"], f["narf_y"], f["narf_z"])
    assert np.array_equal(np.asarray(kp, np.int64), f["narf"])
