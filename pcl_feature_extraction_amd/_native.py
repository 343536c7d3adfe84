"""ctypes binding of libpfx.so (the HIP C-ABI declared in include/pfx.h).

There is deliberately no CPU fallback: if the in-tree ``libpfx.so`` is missing or cannot be
loaded, every entry point raises.  Build it with ``make -C pcl_feature_extraction_amd/csrc``
or ``python -c "import __graft_entry__ as g; g.build()"``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PFX_LIB") or os.path.join(_HERE, "libpfx.so")

PFX_OK, PFX_ERR_INVALID, PFX_ERR_DEVICE, PFX_ERR_CAPACITY, PFX_ERR_UNSUPPORTED = 0, 1, 2, 3, 4
_ERRNAMES = {1: "PFX_ERR_INVALID", 2: "PFX_ERR_DEVICE", 3: "PFX_ERR_CAPACITY", 4: "PFX_ERR_UNSUPPORTED"}

c_f32p = ctypes.POINTER(ctypes.c_float)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_vp = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_dbl = ctypes.c_double
c_int = ctypes.c_int


class NarfParams(ctypes.Structure):
    """pfx_narf_params (NarfKeypoint::Parameters + RangeImageBorderExtractor::Parameters)."""
    _fields_ = [
        ("support_size", ctypes.c_float),
        ("max_no_of_interest_points", ctypes.c_int32),
        ("min_distance_between_interest_points", ctypes.c_float),
        ("optimal_distance_to_high_surface_change", ctypes.c_float),
        ("min_interest_value", ctypes.c_float),
        ("min_surface_change_score", ctypes.c_float),
        ("do_non_maximum_suppression", ctypes.c_int32),
        ("calculate_sparse_interest_image", ctypes.c_int32),
        ("no_of_polynomial_approximations_per_point", ctypes.c_int32),
        ("add_points_on_straight_edges", ctypes.c_int32),
        ("pixel_radius_borders", ctypes.c_int32),
        ("pixel_radius_plane_extraction", ctypes.c_int32),
        ("pixel_radius_border_direction", ctypes.c_int32),
        ("minimum_border_probability", ctypes.c_float),
        ("pixel_radius_principal_curvature", ctypes.c_int32),
    ]


class Camera(ctypes.Structure):
    """pfx_camera (RangeImagePlanar::createFromPointCloudWithFixedSize arguments)."""
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("center_x", ctypes.c_float), ("center_y", ctypes.c_float),
        ("focal_length_x", ctypes.c_float), ("focal_length_y", ctypes.c_float),
        ("sensor_pose", ctypes.c_float * 16),
        ("coordinate_frame", ctypes.c_int32),
        ("noise_level", ctypes.c_float), ("min_range", ctypes.c_float),
    ]


class PcdHeader(ctypes.Structure):
    _fields_ = [
        ("points", ctypes.c_int64), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("data", ctypes.c_int32), ("point_size", ctypes.c_int32),
        ("x_offset", ctypes.c_int32), ("y_offset", ctypes.c_int32), ("z_offset", ctypes.c_int32),
        ("nfields", ctypes.c_int32), ("viewpoint", ctypes.c_float * 7), ("data_offset", ctypes.c_int64),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "pfx_narf_params_default": (None, [ctypes.POINTER(NarfParams)]),
    "pfx_camera_default": (None, [ctypes.POINTER(Camera)]),
    "pfx_ctx_create": (c_int, [c_int, ctypes.POINTER(c_vp)]),
    "pfx_ctx_destroy": (None, [c_vp]),
    "pfx_last_error": (ctypes.c_char_p, [c_vp]),
    "pfx_ctx_set_stream": (c_int, [c_vp, c_vp]),
    "pfx_ctx_use_own_stream": (c_int, [c_vp]),
    "pfx_ctx_get_stream": (c_vp, [c_vp]),
    "pfx_ctx_synchronize": (c_int, [c_vp]),
    "pfx_ctx_trim": (c_int, [c_vp]),
    "pfx_ctx_set_timing": (c_int, [c_vp, c_int]),
    "pfx_ctx_set_shared": (c_int, [c_vp, c_int]),
    "pfx_ctx_reset_timing": (c_int, [c_vp]),
    "pfx_ctx_kernel_time": (c_int, [c_vp, ctypes.c_char_p, ctypes.POINTER(c_dbl), c_i64p]),
    "pfx_ctx_last_stats": (c_int, [c_vp, ctypes.c_char_p, c_i64p]),
    "pfx_radius_search": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_dbl,
                                  c_vp, c_vp, c_vp, c_i64]),
    "pfx_normals": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pfx_normals_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pfx_normals_fast": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pfx_normals_fast_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pfx_fpfh": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                         c_int, c_dbl, c_vp]),
    "pfx_fpfh_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                             c_i64, c_int, c_dbl, c_vp]),
    "pfx_fpfh_after_normals_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                           c_i64, c_int, c_dbl, c_vp]),
    "pfx_fpfh_prepare_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl]),
    "pfx_fpfh_support_mask_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp]),
    "pfx_fpfh_support_ball_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp]),
    "pfx_fpfh_prepare_queries_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_dbl]),
    "pfx_normals_lists_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp]),
    "pfx_normals_prepare_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl]),
    "pfx_normals_launch_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pfx_normals_finish_dev": (c_int, [c_vp, c_vp]),
    "pfx_normals_gate_dev": (c_int, [c_vp, c_vp]),
    "pfx_normals_grid_launch_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl]),
    "pfx_normals_subset_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, ctypes.c_int32, c_vp, c_vp, c_vp,
                                       c_vp, c_vp]),
    "pfx_normals_chains_dev": (c_int, [c_vp, c_vp, c_vp, ctypes.c_int32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pfx_shot": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                         c_dbl, c_vp, c_vp]),
    "pfx_shot_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                             c_i64, c_dbl, c_vp, c_vp]),
    "pfx_range_image_planar": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(Camera), c_vp]),
    "pfx_narf_keypoints": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(Camera),
                                   ctypes.POINTER(NarfParams), c_vp, c_i64, c_i64p]),
    "pfx_narf_keypoints_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(Camera),
                                       ctypes.POINTER(NarfParams), c_vp, c_i64, c_i64p]),
    "pfx_narf_debug_image": (c_int, [c_vp, ctypes.c_char_p, c_vp, c_i64]),
    "pfx_gather_points_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp,
                                      c_i64, c_i64p]),
    "pfx_nearest_descriptors_dev": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, ctypes.c_int32,
                                            c_vp, c_vp, c_vp, c_vp]),
    "pfx_pcd_read_header": (c_int, [ctypes.c_char_p, ctypes.POINTER(PcdHeader)]),
    "pfx_pcd_load_xyz_dev": (c_int, [c_vp, ctypes.c_char_p, c_vp, c_vp, c_vp, c_i64, c_i64p,
                                     ctypes.POINTER(PcdHeader)]),
    "pfx_nearest_descriptors": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, ctypes.c_int32, c_vp, c_vp]),
    "pfx_correspondences_dev": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, ctypes.c_int32,
                                        c_vp, c_vp, c_i64, c_i64p]),
    "pfx_correspondences": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, ctypes.c_int32,
                                    c_vp, c_vp, c_i64, c_i64p]),
    "pfx_cloud_resolution_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(ctypes.c_double)]),
    "pfx_cloud_resolution": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(ctypes.c_double)]),
    "pfx_iss_keypoints_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_int32, ctypes.c_double, ctypes.c_double, c_vp, c_i64, c_i64p, c_vp]),
    "pfx_iss_keypoints": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double, ctypes.c_int32,
                                  ctypes.c_double, ctypes.c_double, c_vp, c_i64, c_i64p, c_vp]),
    "pfx_harris3d_keypoints_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_float,
                                           ctypes.c_int32, ctypes.c_int32, c_vp, c_i64, c_i64p, c_vp, c_vp, c_i64p,
                                           c_vp]),
    "pfx_harris3d_keypoints": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_float,
                                       ctypes.c_int32, ctypes.c_int32, c_vp, c_i64, c_i64p, c_vp, c_vp, c_i64p, c_vp]),
    "pfx_harris6d_keypoints_dev": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_float,
                                           ctypes.c_int32, ctypes.c_int32, c_vp, c_i64, c_i64p, c_vp, c_vp, c_i64p,
                                           c_vp, c_vp]),
    "pfx_harris6d_keypoints": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_float,
                                       ctypes.c_int32, ctypes.c_int32, c_vp, c_i64, c_i64p, c_vp, c_vp, c_i64p, c_vp,
                                       c_vp]),
    "pfx_batch_create": (c_int, [c_vp, c_int, ctypes.POINTER(c_vp)]),
    "pfx_batch_plan": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "pfx_batch_destroy": (None, [c_vp]),
    "pfx_batch_last_error": (ctypes.c_char_p, [c_vp]),
    "pfx_batch_narf_fpfh": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(Camera),
                                    ctypes.POINTER(NarfParams), c_dbl, c_dbl, c_vp, c_vp, c_i64, c_vp]),
    "pfx_ransac_rejector": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                    ctypes.c_double, ctypes.c_int32, c_vp, c_i64p, c_vp]),
}

_lib = None


class PfxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


def lib():
    """Load libpfx.so (raises OSError if it is missing: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built: run `make -C {os.path.join(_HERE, 'csrc')}`")
        # One HIP runtime per process: torch wheels ship their own libamdhip64 (SONAME
        # libamdhip64.so.7, but torch's NEEDED entry is the unversioned name).  Loading torch first
        # makes libpfx's NEEDED libamdhip64.so.7 bind to that copy; the other order would load two
        # runtimes and torch would find no GPU (and stream handles could not be shared).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lb = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lb, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lb
    return _lib


def exported_symbols():
    return sorted(_SIGS)
