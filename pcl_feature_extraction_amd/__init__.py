"""pcl_feature_extraction_amd -- MI355X-native (gfx950) hot path of srv/pcl_feature_extraction.

NARF keypoints on the planar range image + normals + FPFH-33 / SHOT-352 descriptors over radius
neighbourhoods, as hand-written HIP kernels behind the C-ABI in include/pfx.h (libpfx.so).
See DESIGN.md.
"""
from ._native import PfxError, lib  # noqa: F401
from .api import Batch, Context, camera, narf_params  # noqa: F401

__all__ = ["Batch", "Context", "PfxError", "camera", "narf_params", "lib"]
