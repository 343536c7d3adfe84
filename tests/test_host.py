"""Host-side pieces (CPU only): PCD I/O, the synthetic scan generators, pipeline helpers."""
import os

import numpy as np
import pytest

from pcl_feature_extraction_amd.pcd import read_pcd, write_pcd
from pcl_feature_extraction_amd.pipeline import keypoint_rows
from pcl_feature_extraction_amd.synth import synth_room, synth_seabed

CLOUDS = os.path.join(os.path.dirname(__file__), "golden", "clouds")


@pytest.mark.parametrize("name", ["indoor_source", "indoor_target", "underwater_source", "underwater_target"])
def test_reference_clouds_parse(name):
    c = read_pcd(os.path.join(CLOUDS, name + ".pcd"))
    assert c.n > 10_000
    # binary PCD of PCL 1.7: 4096-byte header page + 16 B per point
    assert os.path.getsize(os.path.join(CLOUDS, name + ".pcd")) == 4096 + 16 * c.n
    assert np.isfinite(c.x).all() and np.isfinite(c.y).all() and np.isfinite(c.z).all()


def test_pcd_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    x, y, z = (rng.normal(size=1000).astype(np.float32) for _ in range(3))
    x[3] = np.nan
    p = str(tmp_path / "t.pcd")
    write_pcd(p, x, y, z)
    c = read_pcd(p)
    for a, b in ((c.x, x), (c.y, y), (c.z, z)):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_synth_generators_project_into_the_image():
    for gen, n in ((synth_room, 50_000), (synth_seabed, 50_000)):
        x, y, z, rgb = gen(n, 1)
        assert len(x) == n and np.isfinite(x).all() and (z > 0).all()
        u = 320 + 525 * x / z
        v = 240 + 525 * y / z
        assert (u >= -0.5).all() and (u < 640.5).all() and (v >= -0.5).all() and (v < 480.5).all()


def test_synth_room_density_matches_indoor():
    """k(0.05) ~ 230 (+-15 %) at N = 1e5 (data/indoor: ~233)."""
    import oracle_lib as O
    x, y, z, _ = synth_room(100_000, 1)
    q = np.arange(0, len(x), 50)
    c, _, _ = O.radius_search(x, y, z, x[q], y[q], z[q], 0.05)
    assert 195 <= c.mean() <= 265


def test_keypoint_rows_guards_the_index_quirk():
    # keypoints.h:229 uses a pixel index as a cloud index; indices past the cloud are dropped
    assert list(keypoint_rows(np.array([3, 10, 99]), 50)) == [3, 10]
