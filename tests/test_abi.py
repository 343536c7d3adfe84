"""C-ABI library checks that run without a GPU: libpfx.so loads, exports every symbol that
include/pfx.h declares, and fails loudly (no silent CPU fallback) when no device exists."""
import os
import re

import pytest

from pcl_feature_extraction_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "pfx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pfx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_boundary():
    names = _declared()
    for must in ("pfx_normals", "pfx_fpfh", "pfx_shot", "pfx_narf_keypoints", "pfx_radius_search",
                 "pfx_range_image_planar", "pfx_ctx_create", "pfx_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(_declared()) == sorted(N.exported_symbols())


def test_defaults_match_reference_setup():
    import ctypes
    from pcl_feature_extraction_amd import camera, narf_params
    p = narf_params()
    assert abs(p.support_size - 0.2) < 1e-7                         # keypoints.h:223
    assert p.min_interest_value == pytest.approx(0.45)
    assert p.pixel_radius_borders == 3 and p.minimum_border_probability == pytest.approx(0.8)
    c = camera()
    assert (c.width, c.height) == (640, 480)                         # keypoints.h:204
    assert (c.center_x, c.center_y, c.focal_length_x, c.focal_length_y) == (320.0, 240.0, 525.0, 525.0)
    assert [c.sensor_pose[i] for i in range(16)] == [1.0 if i % 5 == 0 else 0.0 for i in range(16)]
    del ctypes


def test_no_device_is_an_error_not_a_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from pcl_feature_extraction_amd import Context, PfxError
    with pytest.raises(PfxError):
        Context(0)
