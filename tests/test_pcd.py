"""PCD header parsing through the C-ABI (host only; pfx_pcd_read_header) against the Python
reader on the reference's own data files and on ascii / mixed-field binary files."""
import os

import pytest

from pcd_cases import cloud, write_ascii, write_binary_mixed
from pcl_feature_extraction_amd import PfxError
from pcl_feature_extraction_amd.api import pcd_header
from pcl_feature_extraction_amd.pcd import read_pcd

CLOUDS = os.path.join(os.path.dirname(__file__), "golden", "clouds")


@pytest.mark.parametrize("name", ["indoor_source", "indoor_target", "underwater_source", "underwater_target"])
def test_reference_cloud_headers(name):
    path = os.path.join(CLOUDS, name + ".pcd")
    h = pcd_header(path)
    c = read_pcd(path)
    assert h.points == c.n and h.width == c.width and h.height == c.height
    assert h.data == 1 and h.point_size == 16 and (h.x_offset, h.y_offset, h.z_offset) == (0, 4, 8)
    assert tuple(h.viewpoint) == c.viewpoint
    assert h.data_offset + 16 * h.points <= os.path.getsize(path)


def test_ascii_and_mixed_headers(tmp_path):
    x, y, z = cloud(50, 1)
    a, b = tmp_path / "a.pcd", tmp_path / "b.pcd"
    write_ascii(a, x, y, z)
    write_binary_mixed(b, x, y, z)
    ha, hb = pcd_header(a), pcd_header(b)
    assert (ha.data, ha.point_size, ha.x_offset, ha.y_offset, ha.z_offset) == (0, 4, 0, 1, 2)
    assert tuple(ha.viewpoint) == (1, 2, 3, 1, 0, 0, 0)
    assert (hb.data, hb.point_size, hb.x_offset, hb.y_offset, hb.z_offset) == (1, 19, 15, 7, 3)


def test_header_errors(tmp_path):
    with pytest.raises(PfxError):
        pcd_header(tmp_path / "missing.pcd")
    p = tmp_path / "d.pcd"
    p.write_text("FIELDS x y z\nSIZE 8 8 8\nTYPE F F F\nWIDTH 1\nPOINTS 1\nDATA ascii\n1 2 3\n")
    with pytest.raises(PfxError):
        pcd_header(p)  # double coordinates: not PointXYZRGB's float32 layout
