"""ctypes binding of include/rtw.h (lib/librtw.so).

This is the reference-side binding a Python caller uses; it mirrors the
structs of rtw.h field for field.  There is no fallback: if librtw.so is
missing, importing the package raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "librtw.so")
# profiling only (tools/exp_cost.sh): an alternate build of the same library
LIB_PATH = os.environ.get("RTW_LIB_OVERRIDE", LIB_PATH)

RTW_OK = 0
RTW_E_INVALID, RTW_E_DEVICE, RTW_E_NO_LIGHTS, RTW_E_NO_SCENE, RTW_E_UNSUPPORTED, RTW_E_PANIC = -1, -2, -3, -4, -5, -6
RTW_F32, RTW_F64 = 0, 1
RTW_LAMBERTIAN, RTW_METAL, RTW_DIELECTRIC, RTW_INVISIBLE, RTW_DIFFUSE_LIGHT = 0, 1, 2, 3, 4
RTW_ACCEL_AUTO, RTW_ACCEL_BRUTE, RTW_ACCEL_BVH = 0, 1, 2
RTW_TEX_SOLID, RTW_TEX_CHECKER, RTW_TEX_NOISE = 0, 1, 2
RTW_LIGHT_SPHERE, RTW_LIGHT_QUAD, RTW_LIGHT_DEFAULT = 0, 1, 2
RTW_LIGHTS_BVH_LEAF = 1

_f64p = C.POINTER(C.c_double)
_u32p = C.POINTER(C.c_uint32)
_f32p = C.POINTER(C.c_float)


class rtw_camera_builder(C.Structure):
    _fields_ = [
        ("has_aspect_ratio", C.c_int32), ("has_image_width", C.c_int32),
        ("has_image_height", C.c_int32), ("aspect_ratio", C.c_double),
        ("image_width", C.c_uint32), ("image_height", C.c_uint32),
        ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32),
        ("background", C.c_double * 3), ("vfov", C.c_double),
        ("lookfrom", C.c_double * 3), ("lookat", C.c_double * 3), ("vup", C.c_double * 3),
        ("defocus_angle", C.c_double), ("focus_dist", C.c_double),
    ]


class rtw_camera(C.Structure):
    _fields_ = [
        ("image_width", C.c_uint32), ("image_height", C.c_uint32),
        ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32),
        ("background", C.c_double * 3), ("defocus_angle", C.c_double),
        ("center", C.c_double * 3), ("pixel00_loc", C.c_double * 3),
        ("pixel_delta_u", C.c_double * 3), ("pixel_delta_v", C.c_double * 3),
        ("defocus_disk_u", C.c_double * 3), ("defocus_disk_v", C.c_double * 3),
    ]


class rtw_scene(C.Structure):
    _fields_ = [
        ("n_spheres", C.c_uint32), ("spheres", _f64p), ("sphere_mat", _u32p),
        ("n_planes", C.c_uint32), ("planes", _f64p), ("plane_mat", _u32p),
        ("n_materials", C.c_uint32), ("mat_type", _u32p), ("mat_params", _f64p),
        ("n_lights", C.c_uint32), ("lights", _f64p),
        ("n_quads", C.c_uint32), ("quads", _f64p), ("quad_mat", _u32p),
        ("n_light_quads", C.c_uint32), ("light_quads", _f64p), ("light_kinds", _u32p),
        ("n_boxes", C.c_uint32), ("boxes", _f64p), ("box_mat", _u32p),
        ("mat_tex", _u32p), ("n_textures", C.c_uint32), ("tex_type", _u32p), ("tex_params", _f64p),
        ("tex_refs", _u32p), ("n_perlin", C.c_uint32), ("perlin_vec", _f64p), ("perlin_perm", _u32p),
        ("n_light_other", C.c_uint32), ("light_flags", C.c_uint32),
    ]


ABI_VERSION = 10    # RTW_ABI_VERSION of include/rtw.h


class rtw_stats(C.Structure):
    _fields_ = [
        ("samples", C.c_uint64), ("segments", C.c_uint64), ("lambertian", C.c_uint64),
        ("kernel_ms", C.c_double), ("accel", C.c_uint32), ("chunk", C.c_uint32),
        ("node_visits", C.c_uint64), ("sphere_tests", C.c_uint64),
        ("bvh_width", C.c_uint32), ("kernel", C.c_uint32),
        ("panic_plane_uv", C.c_uint64), ("panic_no_lights", C.c_uint64),
        ("light_tests", C.c_uint64), ("grid_cells", C.c_uint64),
    ]


# (name, restype, argtypes) for every entry point declared in include/rtw.h
PROTOTYPES = [
    ("rtw_abi_version", C.c_int, []),
    ("rtw_create", C.c_void_p, [C.c_int, C.c_int]),
    ("rtw_create_devices", C.c_int, [C.POINTER(C.c_int), C.c_uint32, C.c_int, C.POINTER(C.c_void_p)]),
    ("rtw_create_mask", C.c_void_p, [C.c_uint64, C.c_int]),
    ("rtw_create_mask_ex", C.c_int, [C.c_uint64, C.c_int, C.POINTER(C.c_void_p)]),
    ("rtw_visible_devices", C.c_int, []),
    ("rtw_create_virtual", C.c_int, [C.c_int, C.c_uint32, C.c_int, C.POINTER(C.c_void_p)]),
    ("rtw_device_count", C.c_uint32, [C.c_void_p]),
    ("rtw_device_ctx", C.c_void_p, [C.c_void_p, C.c_uint32]),
    ("rtw_device_of", C.c_int, [C.c_void_p]),
    ("rtw_destroy", None, [C.c_void_p]),
    ("rtw_last_error", C.c_char_p, [C.c_void_p]),
    ("rtw_precision", C.c_int, [C.c_void_p]),
    ("rtw_set_chunk", C.c_int, [C.c_void_p, C.c_uint32]),
    ("rtw_set_accel", C.c_int, [C.c_void_p, C.c_int]),
    ("rtw_set_tuning", C.c_int, [C.c_void_p, C.c_char_p, C.c_int64]),
    ("rtw_camera_build", C.c_int, [C.POINTER(rtw_camera_builder), C.POINTER(rtw_camera)]),
    ("rtw_camera_builder_default", None, [C.POINTER(rtw_camera_builder)]),
    ("rtw_set_scene", C.c_int, [C.c_void_p, C.POINTER(rtw_scene)]),
    ("rtw_render", C.c_int, [C.c_void_p, C.POINTER(rtw_camera), C.POINTER(rtw_scene), C.c_uint64,
                             _f64p, C.POINTER(rtw_stats)]),
    ("rtw_render_image_device", C.c_int, [C.c_void_p, C.POINTER(rtw_camera), C.c_uint64, C.c_void_p,
                                          C.c_size_t, C.c_void_p]),
    ("rtw_render_device", C.c_int, [C.c_void_p, C.POINTER(rtw_camera), C.c_uint64, C.c_uint32,
                                    C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p]),
    ("rtw_tile_size", C.c_uint32, []),
    ("rtw_tiles_for_rank", C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("rtw_assemble_tiles", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32,
                                     C.c_uint32, C.c_void_p, C.c_void_p]),
    ("rtw_split_deal", C.c_int, [_u32p, C.c_uint32, C.c_uint32, C.c_uint32, _u32p]),
    ("rtw_set_split", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p]),
    ("rtw_get_split", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, _u32p]),
    ("rtw_tile_costs", C.c_int, [C.c_void_p, C.POINTER(rtw_camera), C.c_uint32, C.c_uint32, _u32p]),
    ("rtw_get_stats", C.c_int, [C.c_void_p, C.POINTER(rtw_stats)]),
    ("rtw_get_stats_rank", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(rtw_stats)]),
    ("rtw_get_timings", C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int]),
    ("rtw_last_kernel", C.c_int, [C.c_void_p]),
    ("rtw_scene_simple", C.c_void_p, [C.c_uint64, C.c_int]),
    ("rtw_world_scene", C.POINTER(rtw_scene), [C.c_void_p]),
    ("rtw_world_camera_builder", None, [C.c_void_p, C.POINTER(rtw_camera_builder)]),
    ("rtw_world_free", None, [C.c_void_p]),
    ("rtw_scene_named", C.c_void_p, [C.c_char_p, C.c_uint64]),
    ("rtw_perlin_generate", C.c_int, [C.c_uint64, _f64p, _u32p]),
    ("rtw_encode_rgb8", C.c_int, [_f64p, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_uint8)]),
    ("rtw_write_ppm", C.c_int, [C.c_char_p, _f64p, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("rtw_encode_rgb8_f32", C.c_int, [_f32p, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_uint8)]),
    ("rtw_write_ppm_f32", C.c_int, [C.c_char_p, _f32p, C.c_uint32, C.c_uint32, C.c_uint32]),
]

_lib = None


def load():
    """Load librtw.so (built by __graft_entry__.build / csrc/Makefile)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so
    # (SONAME libamdhip64.so.7).  Loading torch first lets librtw.so's
    # libamdhip64.so.7 dependency resolve to that same copy; loading librtw.so
    # first would map ROCm's copy too, and the two runtimes then fight over
    # the device (and torch tensors' device pointers would not be valid in ours).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rtw_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {lib.rtw_abi_version()}, this mirror expects "
                          f"{ABI_VERSION}: rebuild it")
    _lib = lib
    return lib
