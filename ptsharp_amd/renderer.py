"""Host-side mirror of PTSharp's Renderer and Buffer (PTSharpCore/Renderer.cs,
Buffer.cs) driving the MI355X path through libptsharp_hip.so.

`Renderer.NewRenderer(scene, camera, sampler, w, h, multithreaded)` keeps the
reference's factory and knobs (SamplesPerPixel, StratifiedSampling, ...);
`RenderParallel()` is one GPU pass; `IterativeRender(pathTemplate, iter)` runs
`iter` passes and writes a PNG after each, as Renderer.cs:702-765 does.  The
Welford state stays in HBM between passes; `Renderer.PBuffer` is refreshed
from it on demand.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import struct
import time
import zlib
from enum import IntEnum

import numpy as np

from . import _abi
from .geometry import Colour
from .scene import Camera, DefaultSampler, Scene

TILE = 32


class Channel(IntEnum):  # Buffer.cs:8-16
    ColorChannel = 0
    VarianceChannel = 1
    StandardDeviationChannel = 2
    SamplesChannel = 3
    AlbedoChannel = 4
    NormalChannel = 5


def tiles_for_rank(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """Static interleaved 32x32 tile ownership: tile t belongs to rank t % world."""
    n = ((width + TILE - 1) // TILE) * ((height + TILE - 1) // TILE)
    return np.arange(rank, n, world, dtype=np.int32)


class Buffer:
    """PTSharpCore.Buffer: per-pixel Welford {Samples, M, V} (Buffer.cs:18-97), held as
    arrays M,V [H,W,3] float64 and N [H,W] int32 (row-major, like pt_read_buffer)."""

    def __init__(self, w: int, h: int):
        self.W, self.H = w, h
        self.M = np.zeros((h, w, 3), np.float64)
        self.V = np.zeros((h, w, 3), np.float64)
        self.N = np.zeros((h, w), np.int32)

    def Samples(self, x, y) -> int:
        return int(self.N[y, x])

    def Color(self, x, y) -> Colour:
        return Colour(*self.M[y, x])

    def Variance(self, x, y) -> Colour:
        n = self.N[y, x]
        if n < 2:
            return Colour(0, 0, 0)
        return Colour(*(self.V[y, x] / (n - 1)))

    def StandardDeviation(self, x, y) -> Colour:
        return self.Variance(x, y).Pow(float(np.float32(0.5)))

    def Image(self, channel: Channel = Channel.ColorChannel) -> np.ndarray:
        """Buffer.Image (Buffer.cs:134-202) as an [H,W,3] uint8 array."""
        if channel == Channel.ColorChannel:
            with np.errstate(invalid="ignore"):
                c = np.power(self.M, 1.0 / 2.2)
        elif channel == Channel.VarianceChannel:
            n = self.N[..., None].astype(np.float64)
            c = np.where(n >= 2, self.V / np.maximum(n - 1, 1), 0.0)
        elif channel == Channel.StandardDeviationChannel:
            n = self.N[..., None].astype(np.float64)
            c = np.power(np.where(n >= 2, self.V / np.maximum(n - 1, 1), 0.0), float(np.float32(0.5)))
        elif channel == Channel.SamplesChannel:
            mx = max(int(self.N.max()), 1)
            c = np.repeat((self.N / mx)[..., None], 3, axis=2)
        else:
            raise ValueError(f"channel {channel} is outside the render path (albedo/normal heuristics)")
        with np.errstate(invalid="ignore"):
            v = np.clip(c * 255, 0, 255)
        v = np.nan_to_num(v, nan=0.0)
        return v.astype(np.uint8)  # (byte) truncates toward zero


def write_png(path: str, rgb: np.ndarray) -> None:
    """Minimal PNG (8-bit RGB) writer — stands in for SkiaSharp's encoder (Renderer.cs:723-729)."""
    h, w, _ = rgb.shape
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


class Renderer:
    """PTSharpCore.Renderer on the MI355X path."""

    PBuffer: Buffer = None  # static, as Renderer.PBuffer (Renderer.cs:20)

    def __init__(self):
        self.Scene: Scene = None
        self.Camera: Camera = None
        self.Sampler: DefaultSampler = None
        self.SamplesPerPixel = 2
        self.StratifiedSampling = False
        self.AdaptiveSamples = 0
        self.FireflySamples = 0
        self.Denoise = False
        self.NumCPU = 1
        # MI355X extensions (no reference counterpart)
        self.Seed = 0            # Random.Shared is unseedable; this keys the counter-based stream
        self.Device = 0
        self.Tiles = None        # optional 32x32 tile ids this context renders (multi-GPU sharding)
        self.Engine = _abi.ENGINE_AUTO  # scheduling only: both engines compute identical per-ray arithmetic
        self.Flags = 0                  # _abi.PASS_KERNEL_TIMING: per-kernel hipEvent timing in Stats()
        self.Verbose = False
        self._ctx = None
        self._lib = None
        self._uploaded = None
        self._pass = 0
        self.iterations = 0

    @staticmethod
    def NewRenderer(scene: Scene, camera: Camera, sampler: DefaultSampler, w: int, h: int, multithreaded: bool = True,
                    device: int = 0) -> "Renderer":
        r = Renderer()
        r.Scene, r.Camera, r.Sampler = scene, camera, sampler
        r.W, r.H = int(w), int(h)
        r.NumCPU = os.cpu_count() if multithreaded else 1
        r.Device = device
        Renderer.PBuffer = Buffer(r.W, r.H)
        r._lib = _abi.load_library()
        ctx = C.c_void_p()
        opts = _abi.pt_device_opts(device, r.W, r.H)
        _abi.check(r._lib.pt_create(C.byref(opts), C.byref(ctx)), "pt_create")
        r._ctx = ctx
        return r

    def __del__(self):
        self.close()

    def close(self):
        if getattr(self, "_ctx", None) is not None and self._lib is not None:
            self._lib.pt_destroy(self._ctx)
            self._ctx = None

    # ------------------------------------------------------------- passes
    def _ensure_scene(self):
        flat = self.Scene.Compile()  # Scene.Compile (Renderer.cs:208)
        if self._uploaded is not flat:
            _abi.check(self._lib.pt_upload_scene(self._ctx, C.byref(flat.desc)), "pt_upload_scene")
            self._uploaded = flat

    def _pass_params(self, spp=None, pass_index=None):
        tiles = self.Tiles
        if tiles is not None:
            tiles = np.ascontiguousarray(tiles, dtype=np.int32)
            self._tiles_keep = tiles
        pp = _abi.pt_pass_params(int(spp or self.SamplesPerPixel), int(bool(self.StratifiedSampling)),
                                 C.c_uint64(self.Seed & 0xFFFFFFFFFFFFFFFF).value,
                                 int(self._pass if pass_index is None else pass_index),
                                 0 if tiles is None else len(tiles),
                                 C.POINTER(C.c_int32)() if tiles is None else tiles.ctypes.data_as(C.POINTER(C.c_int32)),
                                 int(self.Engine), int(self.Flags), int(self.AdaptiveSamples),
                                 int(self.FireflySamples), 1)
        return pp

    def RenderParallel(self) -> None:
        """One pass of Renderer.RenderParallel (Renderer.cs:199-338) on the GPU."""
        self._ensure_scene()
        self._pass += 1
        cam, smp = self.Camera.to_c(), self.Sampler.to_c()
        pp = self._pass_params()
        t0 = time.perf_counter()
        _abi.check(self._lib.pt_render_pass(self._ctx, C.byref(cam), C.byref(smp), C.byref(pp)), "pt_render_pass")
        if self.Verbose:
            print(f"{self.W} x {self.H}, {self.SamplesPerPixel} spp, MI355X device {self.Device}")
            print("time elapsed:", time.perf_counter() - t0)

    def RenderPasses(self, k: int) -> None:
        """k consecutive RenderParallel passes in one call (pt_pass_params.passes): the Buffer is the
        one k RenderParallel() calls leave, bit for bit; plain passes run as one batch on the GPU."""
        k = int(k)
        if k < 1:
            raise ValueError("k must be >= 1")
        self._ensure_scene()
        cam, smp = self.Camera.to_c(), self.Sampler.to_c()
        pp = self._pass_params(pass_index=self._pass + 1)
        pp.passes = k
        _abi.check(self._lib.pt_render_pass(self._ctx, C.byref(cam), C.byref(smp), C.byref(pp)), "pt_render_pass")
        self._pass += k

    def Render(self) -> None:
        """One pass of Renderer.Render (Renderer.cs:80-198), the NumCPU == 1 twin: the same main
        samples, then per pixel AdaptiveSamples individual samples when its standard deviation
        reaches 1 and FireflySamples when it then exceeds 1 (PT_PASS_SERIAL)."""
        flags = self.Flags
        self.Flags = flags | _abi.PASS_SERIAL
        try:
            self.RenderParallel()
        finally:
            self.Flags = flags

    def RenderCounted(self) -> _abi.pt_trace_counters:
        """One pass with traversal counters (bench roofline accounting)."""
        self._ensure_scene()
        self._pass += 1
        cam, smp = self.Camera.to_c(), self.Sampler.to_c()
        pp = self._pass_params()
        out = _abi.pt_trace_counters()
        _abi.check(self._lib.pt_render_pass_counted(self._ctx, C.byref(cam), C.byref(smp), C.byref(pp), C.byref(out)),
                   "pt_render_pass_counted")
        return out

    def Synchronize(self) -> None:
        _abi.check(self._lib.pt_synchronize(self._ctx), "pt_synchronize")

    def ReadBuffer(self) -> Buffer:
        """Copy the HBM Welford state into Renderer.PBuffer."""
        b = Renderer.PBuffer
        if b is None or b.W != self.W or b.H != self.H:
            b = Renderer.PBuffer = Buffer(self.W, self.H)
        _abi.check(self._lib.pt_read_buffer(self._ctx, b.M.ctypes.data_as(C.POINTER(C.c_double)),
                                            b.V.ctypes.data_as(C.POINTER(C.c_double)),
                                            b.N.ctypes.data_as(C.POINTER(C.c_int32))), "pt_read_buffer")
        return b

    def LoadBuffer(self, buf: Buffer, passes_done: int) -> None:
        """Resume an IterativeRender from a saved Buffer (pt_write_buffer): later passes keep adding
        Welford samples to it, numbered from passes_done + 1 (the random streams are keyed by pass)."""
        M = np.ascontiguousarray(buf.M, np.float64)
        V = np.ascontiguousarray(buf.V, np.float64)
        N = np.ascontiguousarray(buf.N, np.int32)
        _abi.check(self._lib.pt_write_buffer(self._ctx, M.ctypes.data_as(C.POINTER(C.c_double)),
                                             V.ctypes.data_as(C.POINTER(C.c_double)),
                                             N.ctypes.data_as(C.POINTER(C.c_int32))), "pt_write_buffer")
        self._pass = int(passes_done)

    def ReadTiles(self, tiles):
        """The Buffer pixels of 32x32 tiles, packed (pt_read_tiles): M, V [n, 32, 32, 3], N [n, 32, 32],
        row-major inside a tile; pixels outside the image are 0."""
        t = np.ascontiguousarray(tiles, np.int32)
        M = np.zeros((len(t), 32, 32, 3), np.float64)
        V = np.zeros((len(t), 32, 32, 3), np.float64)
        N = np.zeros((len(t), 32, 32), np.int32)
        _abi.check(self._lib.pt_read_tiles(self._ctx, t.ctypes.data_as(C.POINTER(C.c_int32)), len(t),
                                           M.ctypes.data_as(C.POINTER(C.c_double)), V.ctypes.data_as(C.POINTER(C.c_double)),
                                           N.ctypes.data_as(C.POINTER(C.c_int32))), "pt_read_tiles")
        return M, V, N

    def WriteTiles(self, tiles, M, V, N) -> None:
        """Write packed tiles (ReadTiles' layout) into the Buffer (pt_write_tiles)."""
        t = np.ascontiguousarray(tiles, np.int32)
        M = np.ascontiguousarray(M, np.float64)
        V = np.ascontiguousarray(V, np.float64)
        N = np.ascontiguousarray(N, np.int32)
        assert M.size == V.size == 3 * N.size == len(t) * 3 * 1024
        _abi.check(self._lib.pt_write_tiles(self._ctx, t.ctypes.data_as(C.POINTER(C.c_int32)), len(t),
                                            M.ctypes.data_as(C.POINTER(C.c_double)), V.ctypes.data_as(C.POINTER(C.c_double)),
                                            N.ctypes.data_as(C.POINTER(C.c_int32))), "pt_write_tiles")

    def Intersect(self, origins, dirs, flags: int = 0):
        """Scene.Intersect (Scene.cs:75-79) of n rays on the device (pt_intersect): (t [n] float64, 1e9 on
        a miss; kind [n] int32, the pt_shape_kind hit or -1).  flags: _abi.MARCH_LANE / MARCH_WAVE."""
        self._ensure_scene()
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        assert o.shape == d.shape
        t = np.zeros(len(o), np.float64)
        k = np.zeros(len(o), np.int32)
        _abi.check(self._lib.pt_intersect(self._ctx, len(o), o.ctypes.data_as(C.POINTER(C.c_float)),
                                          d.ctypes.data_as(C.POINTER(C.c_float)), int(flags),
                                          t.ctypes.data_as(C.POINTER(C.c_double)), k.ctypes.data_as(C.POINTER(C.c_int32))),
                   "pt_intersect")
        return t, k

    def Occluded(self, origins, dirs, t_max, flags: int = 0) -> np.ndarray:
        """The shadow query after the light's own t (pt_occluded): [n] int32, 1 where a shape is hit
        strictly nearer than t_max."""
        self._ensure_scene()
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        tm = np.ascontiguousarray(t_max, np.float64).reshape(-1)
        assert o.shape == d.shape and len(tm) == len(o)
        b = np.zeros(len(o), np.int32)
        _abi.check(self._lib.pt_occluded(self._ctx, len(o), o.ctypes.data_as(C.POINTER(C.c_float)),
                                         d.ctypes.data_as(C.POINTER(C.c_float)), tm.ctypes.data_as(C.POINTER(C.c_double)),
                                         int(flags), b.ctypes.data_as(C.POINTER(C.c_int32))), "pt_occluded")
        return b

    def ResetBuffer(self) -> None:
        _abi.check(self._lib.pt_reset_buffer(self._ctx), "pt_reset_buffer")
        self._pass = 0

    def Stats(self) -> _abi.pt_stats:
        s = _abi.pt_stats()
        _abi.check(self._lib.pt_stats_get(self._ctx, C.byref(s)), "pt_stats_get")
        return s

    def IterativeRender(self, pathTemplate: str | None, iterations: int) -> np.ndarray:
        """Renderer.IterativeRender (Renderer.cs:702-765).  Each iteration is one Render
        (NumCPU == 1) or RenderParallel pass, including its adaptive / firefly phases."""
        self.iterations = iterations
        img = None
        for i in range(1, iterations + 1):
            if self.Verbose:
                print(f"Iteration {i} of {iterations}")
            if self.NumCPU == 1:  # Renderer.cs:712-719
                self.Render()
            else:
                self.RenderParallel()
            if pathTemplate:
                img = self.ReadBuffer().Image(Channel.ColorChannel)
                write_png(pathTemplate.replace("{0}", str(i)), img)
        if img is None:
            img = self.ReadBuffer().Image(Channel.ColorChannel)
        return img

    # ------------------------------------------------------------- multi-GPU
    def CommInit(self, nranks: int, rank: int, unique_id: bytes) -> None:
        idb = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        _abi.check(self._lib.pt_comm_init(self._ctx, nranks, rank, idb), "pt_comm_init")

    def Gather(self, root: int = 0) -> None:
        _abi.check(self._lib.pt_comm_gather(self._ctx, root), "pt_comm_gather")

    @staticmethod
    def CommInitAll(renderers: list) -> None:
        """One communicator over renderers on distinct devices of this process (pt_comm_init_all)."""
        lib = _abi.load_library()
        arr = (C.c_void_p * len(renderers))(*[r._ctx.value for r in renderers])
        _abi.check(lib.pt_comm_init_all(arr, len(renderers)), "pt_comm_init_all")

    @staticmethod
    def GatherAll(renderers: list, root: int = 0) -> None:
        lib = _abi.load_library()
        arr = (C.c_void_p * len(renderers))(*[r._ctx.value for r in renderers])
        _abi.check(lib.pt_comm_gather_all(arr, len(renderers), root), "pt_comm_gather_all")

    @staticmethod
    def CommUniqueId() -> bytes:
        lib = _abi.load_library()
        buf = (C.c_uint8 * 128)()
        _abi.check(lib.pt_comm_unique_id(buf), "pt_comm_unique_id")
        return bytes(buf)
