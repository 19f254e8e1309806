"""ctypes wrapper of oracle/_build/liboracle.so — the CPU restatement used as the
parity checker and as bench.py's cpu_baseline.  TEST INFRASTRUCTURE ONLY: only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.

The oracle's structs share the C-ABI layouts of include/ptsharp_hip.h, so the
product's host-side flattening (ptsharp_amd.scene.FlatScene) feeds both.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from ptsharp_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

_lib = None


def build_oracle() -> str:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return ORACLE_SO


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        L = C.CDLL(build_oracle())
        vp, f3, i32p = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int32)
        dp = C.POINTER(C.c_double)
        L.or_scene_create.restype = vp
        L.or_scene_create.argtypes = [C.POINTER(_abi.pt_scene_desc)]
        L.or_scene_destroy.argtypes = [vp]
        L.or_scene_tree_nodes.restype = C.c_int64
        L.or_scene_tree_nodes.argtypes = [vp]
        L.or_render_pass.restype = C.c_int64
        L.or_render_pass.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(_abi.pt_camera), C.POINTER(_abi.pt_sampler),
                                     C.POINTER(_abi.pt_pass_params), dp, dp, i32p, C.c_int32, C.c_int32]
        L.or_render_pixels.restype = C.c_int64
        L.or_render_pixels.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(_abi.pt_camera), C.POINTER(_abi.pt_sampler),
                                       C.POINTER(_abi.pt_pass_params), C.c_int64, C.c_int64, C.c_int64, dp, dp, i32p,
                                       C.c_int32]
        L.or_intersect.restype = C.c_double
        L.or_intersect.argtypes = [vp, f3, f3, C.c_int32, i32p, i32p]
        L.or_hit_info.restype = C.c_int32
        L.or_hit_info.argtypes = [vp, f3, f3, f3, f3, i32p, i32p]
        L.or_cast_ray.argtypes = [C.POINTER(_abi.pt_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_double,
                                  C.c_double, C.c_uint64, f3, f3]
        L.or_prim_intersect.restype = C.c_double
        L.or_prim_intersect.argtypes = [C.c_int32, f3, f3, f3, C.c_double, f3, f3]
        L.or_prim_normal.argtypes = [C.c_int32, f3, f3, f3, f3, f3, f3, f3, f3]
        L.or_texture_sample.argtypes = [vp, C.c_int32, C.c_int32, C.c_double, C.c_double, dp]
        L.or_shape_uv.argtypes = [vp, C.c_int32, C.c_int32, f3, f3]
        L.or_environment.argtypes = [vp, f3, dp]
        L.or_hit_surface.restype = C.c_int32
        L.or_hit_surface.argtypes = [vp, f3, f3, dp, dp]
        L.or_sdf_evaluate.restype = C.c_double
        L.or_sdf_evaluate.argtypes = [vp, C.c_int32, f3]
        L.or_volume_sample.restype = C.c_double
        L.or_volume_sample.argtypes = [vp, C.c_int32, C.c_double, C.c_double, C.c_double]
        L.or_shape_box.argtypes = [vp, C.c_int32, C.c_int32, f3, f3]
        L.or_camera_key.restype = C.c_uint64
        L.or_camera_key.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32]
        L.or_child_key.restype = C.c_uint64
        L.or_child_key.argtypes = [C.c_uint64, C.c_uint32]
        L.or_light_key.restype = C.c_uint64
        L.or_light_key.argtypes = [C.c_uint64, C.c_uint32]
        L.or_draw.restype = C.c_double
        L.or_draw.argtypes = [C.c_uint64, C.c_uint32]
        L.or_bounce.restype = C.c_int32
        L.or_bounce.argtypes = [vp, f3, f3, C.c_double, C.c_double, C.c_int32, C.c_uint64, f3, f3, i32p, dp]
        L.or_cone.argtypes = [f3, C.c_double, C.c_double, C.c_double, C.c_uint64, f3]
        L.or_lights.restype = C.c_int32
        L.or_lights.argtypes = [vp, i32p, i32p, C.c_int32]
        L.or_sample_light.restype = C.c_int64
        L.or_sample_light.argtypes = [vp, f3, f3, C.c_int32, C.c_uint64, C.c_int32, dp]
        L.or_sample_lights.restype = C.c_int64
        L.or_sample_lights.argtypes = [vp, f3, f3, C.c_uint64, C.c_int32, C.c_int32, dp]
        L.or_any_nearer.restype = C.c_int32
        L.or_any_nearer.argtypes = [vp, f3, f3, C.c_double]
        _lib = L
    return _lib


def f3(v) -> C.Array:
    return (C.c_float * 3)(*[float(np.float32(x)) for x in v])


class OracleScene:
    def __init__(self, scene):
        self.flat = scene.Compile()
        self.h = lib().or_scene_create(C.byref(self.flat.desc))
        if not self.h:
            raise RuntimeError("or_scene_create failed")

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_scene_destroy(self.h)
            self.h = None

    def intersect(self, origin, direction, brute=False):
        k, i = C.c_int32(), C.c_int32()
        t = lib().or_intersect(self.h, f3(origin), f3(direction), int(brute), C.byref(k), C.byref(i))
        return t, k.value, i.value

    def bounce(self, origin, direction, u, v, btype, key):
        """Ray.Bounce at the nearest hit: (origin, direction, reflected, p) or None on a miss."""
        o, d, refl, p = (C.c_float * 3)(), (C.c_float * 3)(), C.c_int32(), C.c_double()
        if not lib().or_bounce(self.h, f3(origin), f3(direction), u, v, btype, key, o, d, C.byref(refl), C.byref(p)):
            return None
        return tuple(o), tuple(d), bool(refl.value), p.value

    def lights(self):
        k, i = (C.c_int32 * 64)(), (C.c_int32 * 64)()
        n = lib().or_lights(self.h, k, i, 64)
        return [(k[j], i[j]) for j in range(min(n, 64))]

    def sample_light(self, origin, normal, light, key, soft_shadows=True):
        out = (C.c_double * 3)()
        rays = lib().or_sample_light(self.h, f3(origin), f3(normal), light, key, int(soft_shadows), out)
        return tuple(out), rays

    def sample_lights(self, origin, normal, key, light_mode, soft_shadows=True):
        out = (C.c_double * 3)()
        rays = lib().or_sample_lights(self.h, f3(origin), f3(normal), key, int(light_mode), int(soft_shadows), out)
        return tuple(out), rays

    def any_nearer(self, origin, direction, t_light) -> bool:
        return bool(lib().or_any_nearer(self.h, f3(origin), f3(direction), t_light))

    def tree_nodes(self) -> int:
        return lib().or_scene_tree_nodes(self.h)

    def texture_sample(self, texture: int, kind: int, u: float, v: float):
        out = (C.c_double * 3)()
        lib().or_texture_sample(self.h, texture, kind, u, v, out)
        return tuple(out)

    def shape_uv(self, kind: int, index: int, p):
        out = (C.c_float * 3)()
        lib().or_shape_uv(self.h, kind, index, f3(p), out)
        return tuple(out)

    def environment(self, direction):
        out = (C.c_double * 3)()
        lib().or_environment(self.h, f3(direction), out)
        return tuple(out)

    def sdf_evaluate(self, node: int, p) -> float:
        return lib().or_sdf_evaluate(self.h, node, f3(p))

    def volume_sample(self, volume: int, x, y, z) -> float:
        return lib().or_volume_sample(self.h, volume, x, y, z)

    def shape_box(self, kind: int, index: int):
        mn, mx = (C.c_float * 3)(), (C.c_float * 3)()
        lib().or_shape_box(self.h, kind, index, mn, mx)
        return tuple(mn), tuple(mx)

    def hit_surface(self, origin, direction):
        col, gloss = (C.c_double * 3)(), C.c_double()
        if not lib().or_hit_surface(self.h, f3(origin), f3(direction), col, C.byref(gloss)):
            return None
        return tuple(col), gloss.value


def default_threads() -> int:
    """Host threads for the oracle: OMP_NUM_THREADS (16 on the GPU box, whose os.cpu_count() is
    the whole machine's), else the CPUs here, at most 16."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() and int(env) > 0 else min(os.cpu_count() or 1, 16)


def pass_params(spp, seed=0, pass_index=1, stratified=False, tiles=None, adaptive=0, firefly=0, serial=False):
    keep = None
    if tiles is not None:
        keep = np.ascontiguousarray(tiles, np.int32)
    pp = _abi.pt_pass_params(spp, int(stratified), seed, pass_index, 0 if keep is None else len(keep),
                             C.POINTER(C.c_int32)() if keep is None else keep.ctypes.data_as(C.POINTER(C.c_int32)),
                             0, _abi.PASS_SERIAL if serial else 0, int(adaptive), int(firefly))
    pp._keep = keep
    return pp


class OracleBuffer:
    def __init__(self, w, h):
        self.W, self.H = w, h
        self.M = np.zeros((h, w, 3), np.float64)
        self.V = np.zeros((h, w, 3), np.float64)
        self.N = np.zeros((h, w), np.int32)

    def ptrs(self):
        return (self.M.ctypes.data_as(C.POINTER(C.c_double)), self.V.ctypes.data_as(C.POINTER(C.c_double)),
                self.N.ctypes.data_as(C.POINTER(C.c_int32)))


def render(oscene: OracleScene, camera, sampler, w, h, spp, passes=1, seed=0, stratified=False, tiles=None,
           threads=None, brute=False, buf: OracleBuffer = None, first_pass=1, adaptive=0, firefly=0, serial=False):
    """IterativeRender-equivalent on the oracle: `passes` RenderParallel (serial: Render) calls."""
    buf = buf or OracleBuffer(w, h)
    cam, smp = camera.to_c(), sampler.to_c()
    threads = default_threads() if threads is None else threads
    rays = 0
    for p in range(first_pass, first_pass + passes):
        pp = pass_params(spp, seed, p, stratified, tiles, adaptive, firefly, serial)
        rays += lib().or_render_pass(oscene.h, w, h, C.byref(cam), C.byref(smp), C.byref(pp), *buf.ptrs(), threads,
                                     int(brute))
    return buf, rays


def render_pixels(oscene: OracleScene, camera, sampler, w, h, spp, pix_begin, pix_end, pix_stride=1, seed=0,
                  pass_index=1, threads=None, buf: OracleBuffer = None):
    buf = buf or OracleBuffer(w, h)
    cam, smp = camera.to_c(), sampler.to_c()
    threads = default_threads() if threads is None else threads
    pp = pass_params(spp, seed, pass_index)
    rays = lib().or_render_pixels(oscene.h, w, h, C.byref(cam), C.byref(smp), C.byref(pp), pix_begin, pix_end,
                                  pix_stride, *buf.ptrs(), threads)
    return buf, rays
