"""ctypes view of the C-ABI in include/ptsharp_hip.h and the loader for the
in-tree libptsharp_hip.so.

The struct layouts here are the single source of truth on the Python side; the
C# P/Invoke declarations in csharp/HipRenderer.cs mirror the same header.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libptsharp_hip.so")

ABI_VERSION = 9   # PT_ABI_VERSION
PT_OK = 0
PT_ERR_INVALID_ARG = -1
PT_ERR_HIP = -2
PT_ERR_NO_SCENE = -3
PT_ERR_UNSUPPORTED = -4
PT_ERR_OUT_OF_MEMORY = -5
PT_ERR_RCCL = -6
PT_ERR_NO_DEVICE = -7

ENGINE_AUTO, ENGINE_MEGAKERNEL, ENGINE_WAVEFRONT = 0, 1, 2
PASS_KERNEL_TIMING = 1
PASS_SERIAL = 2  # Renderer.Render semantics (Renderer.cs:80-198)
K_CAMERA, K_TRACE, K_SHADE, K_SHADOW, K_FINALIZE, K_MEGAKERNEL, K_ACCUM = range(7)
K_SLOTS = 8   # PT_K_SLOTS

SHAPE_SPHERE, SHAPE_CUBE, SHAPE_PLANE, SHAPE_TRIANGLE, SHAPE_MESH = 0, 1, 2, 3, 4
SHAPE_SDF, SHAPE_VOLUME, SHAPE_TRANSFORMED = 5, 6, 7
MARCH_LANE, MARCH_WAVE = 1, 2   # pt_intersect / pt_occluded flags (PT_MARCH_*)

_f = C.POINTER(C.c_float)
_d = C.POINTER(C.c_double)
_i = C.POINTER(C.c_int32)


class pt_texture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("data", _d)]


class pt_material(C.Structure):
    _fields_ = [("color", C.c_double * 3), ("emittance", C.c_double), ("index", C.c_double),
                ("gloss", C.c_double), ("tint", C.c_double), ("reflectivity", C.c_double),
                ("transparent", C.c_int32), ("texture", C.c_int32), ("normal_texture", C.c_int32),
                ("bump_texture", C.c_int32), ("gloss_texture", C.c_int32), ("_pad", C.c_int32),
                ("bump_multiplier", C.c_double)]


class pt_sdf_node(C.Structure):
    _fields_ = [("op", C.c_int32), ("num_children", C.c_int32), ("first_child", C.c_int32), ("_pad", C.c_int32),
                ("params", C.c_double * 8), ("matrix", C.c_double * 16), ("inverse", C.c_double * 16)]


class pt_sdf_shape(C.Structure):
    _fields_ = [("root", C.c_int32), ("material", C.c_int32)]


class pt_volume_window(C.Structure):
    _fields_ = [("lo", C.c_double), ("hi", C.c_double), ("material", C.c_int32), ("_pad", C.c_int32)]


class pt_volume(C.Structure):
    _fields_ = [("w", C.c_int32), ("h", C.c_int32), ("d", C.c_int32), ("num_windows", C.c_int32),
                ("zscale", C.c_double), ("data", _d), ("windows", C.POINTER(pt_volume_window)),
                ("box_min", C.c_float * 3), ("box_max", C.c_float * 3)]


class pt_transformed_shape(C.Structure):
    _fields_ = [("shape_kind", C.c_int32), ("shape_index", C.c_int32), ("matrix", C.c_double * 16),
                ("inverse", C.c_double * 16)]


class pt_scene_desc(C.Structure):
    _fields_ = [
        ("num_materials", C.c_int32), ("materials", C.POINTER(pt_material)),
        ("num_shapes", C.c_int32), ("shape_kind", _i), ("shape_index", _i),
        ("num_spheres", C.c_int32), ("sphere_center", _f), ("sphere_radius", _d), ("sphere_material", _i),
        ("num_cubes", C.c_int32), ("cube_min", _f), ("cube_max", _f), ("cube_material", _i),
        ("num_planes", C.c_int32), ("plane_point", _f), ("plane_normal", _f), ("plane_material", _i),
        ("num_triangles", C.c_int32), ("tri_v1", _f), ("tri_v2", _f), ("tri_v3", _f),
        ("tri_n1", _f), ("tri_n2", _f), ("tri_n3", _f), ("tri_material", _i),
        ("num_meshes", C.c_int32), ("mesh_first", _i), ("mesh_count", _i),
        ("env_color", C.c_double * 3),
        ("num_textures", C.c_int32), ("textures", C.POINTER(pt_texture)),
        ("tri_t1", _f), ("tri_t2", _f), ("tri_t3", _f),
        ("env_texture", C.c_int32), ("_pad", C.c_int32), ("env_texture_angle", C.c_double),
        ("num_sdf_nodes", C.c_int32), ("sdf_nodes", C.POINTER(pt_sdf_node)), ("sdf_children", _i),
        ("num_sdf_shapes", C.c_int32), ("sdf_shapes", C.POINTER(pt_sdf_shape)),
        ("num_volumes", C.c_int32), ("volumes", C.POINTER(pt_volume)),
        ("num_transformed", C.c_int32), ("transformed", C.POINTER(pt_transformed_shape)),
    ]


class pt_camera(C.Structure):
    _fields_ = [("p", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3), ("w", C.c_float * 3),
                ("m", C.c_double), ("focal_distance", C.c_double), ("aperture_radius", C.c_double)]


class pt_sampler(C.Structure):
    _fields_ = [("first_hit_samples", C.c_int32), ("max_bounces", C.c_int32), ("direct_lighting", C.c_int32),
                ("soft_shadows", C.c_int32), ("light_mode", C.c_int32), ("specular_mode", C.c_int32)]


class pt_pass_params(C.Structure):
    _fields_ = [("spp", C.c_int32), ("stratified", C.c_int32), ("seed", C.c_uint64), ("pass_index", C.c_uint32),
                ("num_tiles", C.c_int32), ("tiles", _i), ("engine", C.c_int32), ("flags", C.c_int32),
                ("adaptive_samples", C.c_int32), ("firefly_samples", C.c_int32), ("passes", C.c_int32)]


class pt_device_opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]


class pt_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("rays_total", C.c_uint64), ("last_pass_ms", C.c_double),
                ("total_ms", C.c_double), ("bvh_nodes", C.c_uint64), ("bvh_bytes", C.c_uint64),
                ("build_ms", C.c_double), ("passes", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("kernel_ms", C.c_double * K_SLOTS), ("kernel_launches", C.c_uint32 * K_SLOTS),
                ("traversal_bytes", C.c_uint64), ("tail_handoffs", C.c_uint64)]


class pt_trace_counters(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("nodes_visited", C.c_uint64), ("prims_tested", C.c_uint64),
                ("shading_fetches", C.c_uint64), ("shadow_rays", C.c_uint64), ("shadow_nodes", C.c_uint64),
                ("shadow_prims", C.c_uint64), ("lit_shadow_rays", C.c_uint64), ("accum_runs", C.c_uint64),
                ("volume_samples", C.c_uint64), ("sdf_evals", C.c_uint64), ("march_clock", C.c_uint64 * 8)]


# name -> (restype, argtypes); every symbol declared in include/ptsharp_hip.h
_f = C.POINTER(C.c_float)


class pt_mesh_data(C.Structure):
    _fields_ = [("num_triangles", C.c_int32)] + [(n, _f) for n in ("v1", "v2", "v3", "n1", "n2", "n3",
                                                                    "t1", "t2", "t3")]


SIGNATURES = {
    "pt_get_version": (C.c_int, []),
    "pt_device_count": (C.c_int, [_i]),
    "pt_create": (C.c_int, [C.POINTER(pt_device_opts), C.POINTER(C.c_void_p)]),
    "pt_upload_scene": (C.c_int, [C.c_void_p, C.POINTER(pt_scene_desc)]),
    "pt_render_pass": (C.c_int, [C.c_void_p, C.POINTER(pt_camera), C.POINTER(pt_sampler), C.POINTER(pt_pass_params)]),
    "pt_synchronize": (C.c_int, [C.c_void_p]),
    "pt_reset_buffer": (C.c_int, [C.c_void_p]),
    "pt_read_buffer": (C.c_int, [C.c_void_p, _d, _d, _i]),
    "pt_write_buffer": (C.c_int, [C.c_void_p, _d, _d, _i]),
    "pt_read_tiles": (C.c_int, [C.c_void_p, _i, C.c_int32, _d, _d, _i]),
    "pt_write_tiles": (C.c_int, [C.c_void_p, _i, C.c_int32, _d, _d, _i]),
    "pt_stats_get": (C.c_int, [C.c_void_p, C.POINTER(pt_stats)]),
    "pt_last_error": (C.c_char_p, []),
    "pt_destroy": (None, [C.c_void_p]),
    "pt_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "pt_comm_init": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_uint8)]),
    "pt_comm_gather": (C.c_int, [C.c_void_p, C.c_int32]),
    "pt_comm_destroy": (C.c_int, [C.c_void_p]),
    "pt_comm_init_all": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32]),
    "pt_comm_gather_all": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.c_int32]),
    "pt_gather_layout": (C.c_int, [C.c_int32, C.c_int32, _i, C.c_int32, C.POINTER(C.c_int64),
                                   C.POINTER(C.c_int64)]),
    "pt_tile_lists_check": (C.c_int, [_i, C.c_int64, C.c_int32]),
    "pt_render_pass_counted": (C.c_int, [C.c_void_p, C.POINTER(pt_camera), C.POINTER(pt_sampler),
                                         C.POINTER(pt_pass_params), C.POINTER(pt_trace_counters)]),
    "pt_scene_bvh_digest": (C.c_int, [C.POINTER(pt_scene_desc), C.POINTER(C.c_uint64)]),
    "pt_intersect": (C.c_int, [C.c_void_p, C.c_int64, _f, _f, C.c_int32, _d, _i]),
    "pt_occluded": (C.c_int, [C.c_void_p, C.c_int64, _f, _f, _d, C.c_int32, _i]),
    "pt_obj_load": (C.c_int, [C.c_char_p, C.POINTER(pt_mesh_data)]),
    "pt_mesh_free": (None, [C.POINTER(pt_mesh_data)]),
    "pt_obj_last_error": (C.c_char_p, []),
    "pt_mesh_smooth_normals": (C.c_int, [C.c_int32, _f, _f, _f, _f, _f, _f]),
}


class PTError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load libptsharp_hip.so.  Raises if it is missing: there is no CPU fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(the HIP render path has no CPU fallback)")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(code: int, where: str) -> None:
    if code != PT_OK:
        msg = load_library().pt_last_error()
        raise PTError(code, where, msg.decode() if msg else "")
