"""GPU: pfx_pcd_load_xyz_dev (loadPCDFile<PointXYZRGB>, evaluation.cpp:226-235) puts exactly the
file's x, y, z into the device SoA arrays: the reference's binary clouds, ascii as savePCDFile
writes it, binary with unaligned fields, NaN points, and the capacity error."""
import os

import numpy as np
import pytest

from pcd_cases import cloud, write_ascii, write_binary_mixed
from pcl_feature_extraction_amd import PfxError
from pcl_feature_extraction_amd.pcd import read_pcd

pytestmark = pytest.mark.gpu
CLOUDS = os.path.join(os.path.dirname(__file__), "golden", "clouds")


def _load(ctx, path, n):
    import torch
    x, y, z = (torch.full((n,), 7.0, device="cuda") for _ in range(3))
    k, h = ctx.pcd_load_xyz_dev(path, x, y, z)
    torch.cuda.synchronize()
    return k, h, x[:k].cpu().numpy(), y[:k].cpu().numpy(), z[:k].cpu().numpy()


def _same(a, b):
    return np.array_equal(np.nan_to_num(a, nan=-9).view(np.uint32), np.nan_to_num(b, nan=-9).view(np.uint32))


@pytest.mark.parametrize("name", ["indoor_source", "underwater_target"])
def test_reference_clouds(ctx, name):
    path = os.path.join(CLOUDS, name + ".pcd")
    c = read_pcd(path)
    k, h, x, y, z = _load(ctx, path, c.n + 5)
    assert k == c.n and tuple(h.viewpoint) == c.viewpoint
    assert _same(x, c.x) and _same(y, c.y) and _same(z, c.z)


def test_ascii_and_unaligned_binary(ctx, tmp_path):
    x, y, z = cloud(3000, 2)
    a, b = str(tmp_path / "a.pcd"), str(tmp_path / "b.pcd")
    write_ascii(a, x, y, z)
    write_binary_mixed(b, x, y, z)
    for p in (a, b):
        k, _, gx, gy, gz = _load(ctx, p, 3000)
        assert k == 3000 and _same(gx, x) and _same(gy, y) and _same(gz, z)


def test_capacity(ctx):
    import torch
    path = os.path.join(CLOUDS, "underwater_source.pcd")
    t = torch.empty(10, device="cuda")
    with pytest.raises(PfxError):
        ctx.pcd_load_xyz_dev(path, t, t, t)
