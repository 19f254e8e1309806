"""Host-side mirror of PTSharp's plugin surface for the render path: Material,
ColorTexture, the IShape kinds the GPU path covers (Sphere, Cube, Plane,
Triangle, Mesh), Scene, Camera and DefaultSampler (PTSharpCore/Material.cs,
Texture.cs, Sphere.cs, Cube.cs, Plane.cs, Triangle.cs, Mesh.cs, Scene.cs,
Camera.cs, Sampler.cs).

`Scene.flatten()` produces the caller-owned arrays of pt_scene_desc
(include/ptsharp_hip.h) — the same flattening the C# HipRenderer performs with
a type switch over Scene.Shapes.
"""
from __future__ import annotations

import ctypes as C
import math
import struct
import zlib
from dataclasses import dataclass, field, replace
from enum import IntEnum

import numpy as np

from . import _abi
from .geometry import Box, Colour, Matrix, Vector, cross_rows, dot_rows, normalize_rows


class LightMode(IntEnum):          # LightMode.cs
    LightModeRandom = 0
    LightModeAll = 1


class SpecularMode(IntEnum):       # SpecularMode.cs
    SpecularModeNaive = 0
    SpecularModeFirst = 1
    SpecularModeAll = 2


def _read_png_rgb8(path: str) -> np.ndarray:
    """Minimal PNG decoder (8-bit grey / grey+alpha / RGB / RGBA / palette, not
    interlaced) standing in for SkiaSharp's decode in Util.LoadImage (Util.cs:57-70).
    Returns [h][w][3] uint8; alpha is dropped (NewTexture reads Red/Green/Blue only)."""
    data = open(path, "rb").read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError(f"{path}: not a PNG file")
    pos, idat, plte = 8, [], None
    w = h = depth = ctype = interlace = None
    while pos < len(data):
        (n,), tag = struct.unpack(">I", data[pos:pos + 4]), data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if tag == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
        elif tag == b"PLTE":
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif tag == b"IDAT":
            idat.append(body)
        elif tag == b"IEND":
            break
    if depth != 8 or interlace != 0 or ctype not in (0, 2, 3, 4, 6):
        raise ValueError(f"{path}: only 8-bit non-interlaced PNG is supported")
    bpp = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8).reshape(h, 1 + w * bpp)
    out = np.zeros((h, w * bpp), np.int32)
    prev = np.zeros(w * bpp, np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:
            cur = line.copy()
            for i in range(w * bpp):
                a = cur[i - bpp] if i >= bpp else 0
                b = prev[i]
                if f == 1:
                    cur[i] = (cur[i] + a) & 255
                elif f == 3:
                    cur[i] = (cur[i] + ((a + b) >> 1)) & 255
                else:
                    c = prev[i - bpp] if i >= bpp else 0
                    pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                    cur[i] = (cur[i] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)) & 255
        out[y], prev = cur, cur
    px = out.astype(np.uint8).reshape(h, w, bpp)
    if ctype == 3:
        return plte[px[:, :, 0]]
    if ctype in (0, 4):
        return np.repeat(px[:, :, :1], 3, axis=2)
    return px[:, :, :3].copy()


class ColorTexture:
    """PTSharpCore.ColorTexture (Texture.cs:96-252): Width x Height fp64 Colour texels,
    row-major (Data[y*Width + x]).  Sampling runs on the GPU (pt_device.h); this host
    object holds the data the C-ABI uploads (pt_texture)."""

    _cache: dict = {}   # ColorTexture.textures (Texture.cs:102)

    def __init__(self, width: int, height: int, data):
        self.Width, self.Height = int(width), int(height)
        self.Data = np.ascontiguousarray(np.asarray(data, np.float64).reshape(self.Height * self.Width, 3))

    @staticmethod
    def NewTexture(rgb8) -> "ColorTexture":
        """ColorTexture.NewTexture (Texture.cs:150-166): Colour(c / 255).Pow(2.2F)."""
        a = np.asarray(rgb8)
        h, w = a.shape[:2]
        gamma = float(np.float32(2.2))   # Pow(2.2F): the float literal widened to double
        return ColorTexture(w, h, (a[:, :, :3].astype(np.float64) / 255) ** gamma)

    @staticmethod
    def LoadTexture(path: str) -> "ColorTexture":
        """ColorTexture.LoadTexture (Texture.cs:134-148) for 8-bit PNG files."""
        return ColorTexture.NewTexture(_read_png_rgb8(path))

    @staticmethod
    def GetTexture(path: str) -> "ColorTexture":
        """ColorTexture.GetTexture (Texture.cs:118-132): cached by path."""
        if path not in ColorTexture._cache:
            ColorTexture._cache[path] = ColorTexture.LoadTexture(path)
        return ColorTexture._cache[path]

    def Pow(self, a: float) -> "ColorTexture":   # ITexture.Pow (Texture.cs:170-177), in place
        self.Data = self.Data ** float(a)
        return self

    def MulScalar(self, a: float) -> "ColorTexture":   # ITexture.MulScalar (Texture.cs:179-186), in place
        self.Data = self.Data * float(a)
        return self


@dataclass(frozen=True)
class Material:
    """PTSharpCore.Material (Material.cs:8-62), texture maps included (§8f row 3)."""
    Color: Colour = field(default_factory=lambda: Colour(0, 0, 0))
    BumpMultiplier: float = 0.0
    Emittance: float = 0.0
    Index: float = 0.0
    Gloss: float = 0.0
    Tint: float = 0.0
    Reflectivity: float = 0.0
    Transparent: bool = False
    Texture: object = None
    NormalTexture: object = None
    BumpTexture: object = None
    GlossTexture: object = None

    def key(self):
        return (self.Color.r, self.Color.g, self.Color.b, self.Emittance, self.Index, self.Gloss, self.Tint,
                self.Reflectivity, bool(self.Transparent), self.BumpMultiplier, id(self.Texture),
                id(self.NormalTexture), id(self.BumpTexture), id(self.GlossTexture))

    # factories (Material.cs:64-97)
    @staticmethod
    def DiffuseMaterial(color: Colour) -> "Material":
        return Material(color, 1, 0, 1, 0, 0, -1, False)

    @staticmethod
    def SpecularMaterial(color: Colour, index: float) -> "Material":
        return Material(color, 1, 0, index, 0, 0, -1, False)

    @staticmethod
    def GlossyMaterial(color: Colour, index: float, gloss: float) -> "Material":
        return Material(color, 1, 0, index, gloss, 0, -1, False)

    @staticmethod
    def ClearMaterial(index: float, gloss: float) -> "Material":
        return Material(Colour(0, 0, 0), 1, 0, index, gloss, 0, -1, True)

    @staticmethod
    def TransparentMaterial(color: Colour, index: float, gloss: float, tint: float) -> "Material":
        return Material(color, 1, 0, index, gloss, tint, -1, True)

    @staticmethod
    def MetallicMaterial(color: Colour, gloss: float, tint: float) -> "Material":
        return Material(color, 1, 0, 1, gloss, tint, 1, False)

    @staticmethod
    def LightMaterial(color: Colour, emittance: float) -> "Material":
        return Material(color, 1, emittance, 1, 0, 0, -1, False)

    def with_(self, **kw) -> "Material":
        return replace(self, **kw)


DEFAULT_MATERIAL = Material()  # `new Material()` / `default` (Mesh.MaterialAt, Mesh.cs:132-135)


class Sphere:
    """PTSharpCore.Sphere (Sphere.cs)."""

    def __init__(self, center: Vector, radius: float, material: Material):
        self.Center, self.Radius, self.Material = center, float(radius), material

    @staticmethod
    def NewSphere(center: Vector, radius: float, material: Material) -> "Sphere":
        return Sphere(center, radius, material)

    def BoundingBox(self) -> Box:
        c, r = self.Center, self.Radius
        return Box(Vector(c.X - r, c.Y - r, c.Z - r), Vector(c.X + r, c.Y + r, c.Z + r))

    def MaterialAt(self, p=None) -> Material:
        return self.Material


class Cube:
    """PTSharpCore.Cube (Cube.cs)."""

    def __init__(self, mn: Vector, mx: Vector, material: Material):
        self.Min, self.Max, self.Material = mn, mx, material

    @staticmethod
    def NewCube(mn: Vector, mx: Vector, material: Material) -> "Cube":
        return Cube(mn, mx, material)

    def BoundingBox(self) -> Box:
        return Box(self.Min, self.Max)

    def MaterialAt(self, p=None) -> Material:
        return self.Material


class Plane:
    """PTSharpCore.Plane (Plane.cs); NewPlane normalises the normal."""

    def __init__(self, point: Vector, normal: Vector, material: Material):
        self.Point, self.Normal, self.Material = point, normal, material

    @staticmethod
    def NewPlane(point: Vector, normal: Vector, material: Material) -> "Plane":
        return Plane(point, normal.Normalize(), material)

    def BoundingBox(self) -> Box:
        return Box(Vector(-1e9, -1e9, -1e9), Vector(1e9, 1e9, 1e9))

    def MaterialAt(self, p=None) -> Material:
        return self.Material


class Triangle:
    """PTSharpCore.Triangle (Triangle.cs), a struct: added to a Scene directly it
    is boxed, so as a light it never passes Sampler's identity test."""

    def __init__(self, v1: Vector, v2: Vector, v3: Vector, n1: Vector = None, n2: Vector = None, n3: Vector = None,
                 material: Material = DEFAULT_MATERIAL, t1: Vector = None, t2: Vector = None, t3: Vector = None):
        self.V1, self.V2, self.V3 = v1, v2, v3
        self.N1 = n1 if n1 is not None else Vector()
        self.N2 = n2 if n2 is not None else Vector()
        self.N3 = n3 if n3 is not None else Vector()
        self.T1 = t1 if t1 is not None else Vector()
        self.T2 = t2 if t2 is not None else Vector()
        self.T3 = t3 if t3 is not None else Vector()
        self.Material = material

    @staticmethod
    def NewTriangle(v1, v2, v3, t1=None, t2=None, t3=None, material: Material = DEFAULT_MATERIAL) -> "Triangle":
        """Triangle.NewTriangle (Triangle.cs:43-55): vertices, texture coordinates, FixNormals."""
        t = Triangle(v1, v2, v3, material=material, t1=t1, t2=t2, t3=t3)
        t.FixNormals()
        return t

    def Normal(self) -> Vector:
        e1 = self.V2.Sub(self.V1)
        e2 = self.V3.Sub(self.V1)
        return e1.Cross(e2).Normalize()

    def FixNormals(self) -> None:  # Triangle.cs:224-237
        n = self.Normal()
        z = Vector()
        if self.N1 == z:
            self.N1 = n
        if self.N2 == z:
            self.N2 = n
        if self.N3 == z:
            self.N3 = n

    def BoundingBox(self) -> Box:
        return Box(self.V1.Min(self.V2).Min(self.V3), self.V1.Max(self.V2).Max(self.V3))

    def MaterialAt(self, p=None) -> Material:
        return self.Material


def fix_normals_arrays(v1, v2, v3, n1, n2, n3):
    """Triangle.FixNormals over arrays: zero normals take the face normal."""
    face = normalize_rows(cross_rows((v2 - v1).astype(np.float32), (v3 - v1).astype(np.float32)))
    out = []
    for n in (n1, n2, n3):
        n = n.copy()
        z = np.all(n == 0, axis=1)
        n[z] = face[z]
        out.append(n)
    return out


class Mesh:
    """PTSharpCore.Mesh (Mesh.cs): a triangle container held as [n,3] float32 arrays
    plus a per-triangle material index into `materials`."""

    def __init__(self, v1, v2, v3, n1, n2, n3, mat_index=None, materials=None, t1=None, t2=None, t3=None):
        self.v1, self.v2, self.v3 = (np.ascontiguousarray(a, dtype=np.float32) for a in (v1, v2, v3))
        self.n1, self.n2, self.n3 = (np.ascontiguousarray(a, dtype=np.float32) for a in (n1, n2, n3))
        n = len(self.v1)
        z = lambda t: np.zeros((n, 3), np.float32) if t is None else np.ascontiguousarray(t, dtype=np.float32)
        self.t1, self.t2, self.t3 = z(t1), z(t2), z(t3)   # Triangle.T1..T3
        self.mat_index = np.zeros(n, np.int32) if mat_index is None else np.asarray(mat_index, np.int32)
        self.materials = list(materials) if materials else [DEFAULT_MATERIAL]

    @staticmethod
    def NewMesh(triangles) -> "Mesh":
        mats, idx = [], []
        for t in triangles:
            if t.Material not in mats:
                mats.append(t.Material)
            idx.append(mats.index(t.Material))
        arr = lambda name: np.array([getattr(t, name).f32() for t in triangles], dtype=np.float32).reshape(-1, 3)
        return Mesh(arr("V1"), arr("V2"), arr("V3"), arr("N1"), arr("N2"), arr("N3"), idx, mats, arr("T1"), arr("T2"),
                    arr("T3"))

    def __len__(self):
        return len(self.v1)

    def copy(self) -> "Mesh":
        return Mesh(self.v1.copy(), self.v2.copy(), self.v3.copy(), self.n1.copy(), self.n2.copy(), self.n3.copy(),
                    self.mat_index.copy(), list(self.materials), self.t1.copy(), self.t2.copy(), self.t3.copy())

    def MaterialAt(self, p=None) -> Material:
        return DEFAULT_MATERIAL

    def SetMaterial(self, material: Material) -> None:
        self.materials = [material]
        self.mat_index = np.zeros(len(self), np.int32)

    def BoundingBox(self) -> Box:
        """Mesh.BoundingBox (Mesh.cs:88-120): component-wise min/max over V1,V2,V3."""
        allv = np.concatenate([self.v1, self.v2, self.v3])
        return Box(Vector(*allv.min(axis=0)), Vector(*allv.max(axis=0)))

    def Transform(self, matrix: Matrix) -> None:
        """Mesh.Transform (Mesh.cs:254-274)."""
        self.v1 = matrix.MulPosition_arrays(self.v1)
        self.v2 = matrix.MulPosition_arrays(self.v2)
        self.v3 = matrix.MulPosition_arrays(self.v3)
        self.n1 = matrix.MulDirection_arrays(self.n1)
        self.n2 = matrix.MulDirection_arrays(self.n2)
        self.n3 = matrix.MulDirection_arrays(self.n3)

    def FitInside(self, box: Box, anchor: Vector) -> None:
        """Mesh.FitInside (Mesh.cs:243-252)."""
        bb = self.BoundingBox()
        scale = box.Size().Div(bb.Size()).MinComponent()
        extra = box.Size().Sub(bb.Size().MulScalar(scale))
        matrix = Matrix.Identity()
        matrix = Matrix.TranslateM(bb.Min.Negate()).Mul(matrix)
        matrix = Matrix.ScaleM(Vector(scale, scale, scale)).Mul(matrix)
        matrix = Matrix.TranslateM(box.Min.Add(extra.Mul(anchor))).Mul(matrix)
        self.Transform(matrix)

    def MoveTo(self, position: Vector, anchor: Vector) -> None:
        m = Matrix.TranslateM(position.Sub(self.BoundingBox().Anchor(anchor)))
        self.Transform(m)

    def SmoothNormals(self) -> None:
        """Mesh.SmoothNormals (Mesh.cs:191-229), natively (pt_mesh_smooth_normals): per
        distinct vertex, the fp32 sum of the corner normals in triangle order, normalised."""
        n = len(self)
        if n == 0:
            return
        lib = _abi.load_library()
        self.n1, self.n2, self.n3 = (np.ascontiguousarray(a, np.float32).copy() for a in (self.n1, self.n2, self.n3))
        f = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(C.POINTER(C.c_float))
        rc = lib.pt_mesh_smooth_normals(n, f(self.v1), f(self.v2), f(self.v3), f(self.n1), f(self.n2), f(self.n3))
        if rc != 0:
            raise _abi.PTError(rc, "pt_mesh_smooth_normals", lib.pt_obj_last_error().decode())


# ---------------------------------------------------------------- SDF.cs (§8f row 4)
class _SDF:
    """A node of an SDF tree (SDF.cs:6-10); evaluated on the GPU (pt_device.h sdf_eval)."""
    op = -1

    def __init__(self, params=(), children=(), matrix=None, inverse=None):
        self.params = tuple(float(x) for x in params)
        self.children = list(children)
        self.matrix, self.inverse = matrix, inverse


class SphereSDF(_SDF):      # SDF.cs:115-140
    op = 0

    @staticmethod
    def NewSphereSDF(radius: float) -> "SphereSDF":
        return SphereSDF((radius, 2))


class CubeSDF(_SDF):        # SDF.cs:142-195
    op = 1

    @staticmethod
    def NewCubeSDF(size: Vector) -> "CubeSDF":
        return CubeSDF(size.f32())


class CylinderSDF(_SDF):    # SDF.cs:197-252
    op = 2

    @staticmethod
    def NewCylinderSDF(radius: float, height: float) -> "CylinderSDF":
        return CylinderSDF((radius, height))


class CapsuleSDF(_SDF):     # SDF.cs:254-285
    op = 3

    @staticmethod
    def NewCapsuleSDF(a: Vector, b: Vector, radius: float) -> "CapsuleSDF":
        return CapsuleSDF(a.f32() + b.f32() + (radius, 2))


class TorusSDF(_SDF):       # SDF.cs:287-319
    op = 4

    @staticmethod
    def NewTorusSDF(major: float, minor: float) -> "TorusSDF":
        return TorusSDF((major, minor, 2, 2))


class TransformSDF(_SDF):   # SDF.cs:321-353
    op = 5

    @staticmethod
    def NewTransformSDF(sdf: _SDF, matrix: Matrix) -> "TransformSDF":
        return TransformSDF((), [sdf], matrix, matrix.Inverse())


class ScaleSDF(_SDF):       # SDF.cs:355-382
    op = 6

    @staticmethod
    def NewScaleSDF(sdf: _SDF, factor: float) -> "ScaleSDF":
        return ScaleSDF((factor,), [sdf])


class UnionSDF(_SDF):       # SDF.cs:384-435
    op = 7

    @staticmethod
    def NewUnionSDF(items) -> "UnionSDF":
        return UnionSDF((), items)


class DifferenceSDF(_SDF):  # SDF.cs:437-477
    op = 8

    @staticmethod
    def NewDifferenceSDF(items) -> "DifferenceSDF":
        return DifferenceSDF((), items)


class IntersectionSDF(_SDF):  # SDF.cs:479-531
    op = 9

    @staticmethod
    def NewIntersectionSDF(items) -> "IntersectionSDF":
        return IntersectionSDF((), items)


class RepeatSDF(_SDF):      # SDF.cs:533-559
    op = 10

    @staticmethod
    def NewRepeaterSDF(sdf: _SDF, step: Vector) -> "RepeatSDF":
        return RepeatSDF(step.f32(), [sdf])


class SDFShape:
    """PTSharpCore.SDFShape (SDF.cs:12-113): a sphere-traced SDF tree with one material."""

    def __init__(self, sdf: _SDF, material: Material):
        self.SDF, self.Material = sdf, material

    @staticmethod
    def NewSDFShape(sdf: _SDF, material: Material) -> "SDFShape":
        return SDFShape(sdf, material)

    def MaterialAt(self, p=None) -> Material:
        return self.Material


class VolumeWindow:
    """Volume.VolumeWindow (Volume.cs:8-19)."""

    def __init__(self, lo: float, hi: float, material: Material):
        self.Lo, self.Hi, self.VolumeWindowMaterial = float(lo), float(hi), material


class Volume:
    """PTSharpCore.Volume (Volume.cs): a W x H x D voxel grid (Data[x + y*W + z*W*H] = red/255)
    marched for iso-windows."""

    def __init__(self, w, h, d, zscale, data, windows, box: Box):
        self.W, self.H, self.D, self.ZScale = int(w), int(h), int(d), float(zscale)
        self.Data = np.ascontiguousarray(np.asarray(data, np.float64).reshape(-1))
        self.Windows = list(windows)
        self.Box = box

    @staticmethod
    def NewVolume(box: Box, images, sliceSpacing: float, windows) -> "Volume":
        """Volume.NewVolume (Volume.cs:48-71): images are [h][w] or [h][w][3+] 8-bit slices (red used)."""
        sl = [np.asarray(im) for im in images]
        sl = [im[:, :, 0] if im.ndim == 3 else im for im in sl]
        h, w = sl[0].shape
        d = len(sl)
        zs = sliceSpacing * d / w
        data = np.stack(sl).astype(np.float64) / 255
        return Volume(w, h, d, zs, data, windows, box)

    def MaterialAt(self, p=None) -> Material:
        """Volume.MaterialAt at the origin, all Scene.Add asks (Volume.cs:148-166); the GPU
        and the oracle evaluate it at every shading point."""
        s = self._sample(0.0, 0.0, 0.0)
        be, bm = float(np.float32(1e9)), DEFAULT_MATERIAL
        for w in self.Windows:
            if w.Lo <= s <= w.Hi:
                return w.VolumeWindowMaterial
            e = min(abs(s - w.Lo), abs(s - w.Hi))
            if e < be:
                be, bm = e, w.VolumeWindowMaterial
        return bm

    def _sample(self, x, y, z):  # Volume.Sample (Volume.cs:73-105), y-from-z slip kept
        z /= self.ZScale
        x = ((x + 1) / 2) * self.W
        y = ((z + 1) / 2) * self.H
        z = ((z + 2) / 2) * self.D
        x0, y0, z0 = math.floor(x), math.floor(y), math.floor(z)
        W, H, D = self.W, self.H, self.D
        get = lambda a, b, c: 0.0 if (a < 0 or b < 0 or c < 0 or a >= W or b >= H or c >= D) else \
            float(self.Data[a + b * W + c * W * H])
        v = {(i, j, k): get(x0 + i, y0 + j, z0 + k) for i in (0, 1) for j in (0, 1) for k in (0, 1)}
        x, y, z = x - x0, y - y0, z - z0
        c00 = v[0, 0, 0] * (1 - x) + v[1, 0, 0] * x
        c01 = v[0, 0, 1] * (1 - x) + v[1, 0, 1] * x
        c10 = v[0, 1, 0] * (1 - x) + v[1, 1, 0] * x
        c11 = v[0, 1, 1] * (1 - x) + v[1, 1, 1] * x
        c0 = c00 * (1 - y) + c10 * y
        c1 = c01 * (1 - y) + c11 * y
        return c0 * (1 - z) + c1 * z


class TransformedShape:
    """PTSharpCore.TransformedShape (TransformedShape.cs), a struct: as a light it never passes
    Sampler's identity test.  The inner shape may be a Sphere, Cube, Plane, SDFShape or Volume."""

    def __init__(self, shape, matrix: Matrix, inverse: Matrix):
        self.Shape, self.Matrix, self.Inverse = shape, matrix, inverse

    @staticmethod
    def NewTransformedShape(shape, matrix: Matrix) -> "TransformedShape":
        return TransformedShape(shape, matrix, matrix.Inverse())

    def MaterialAt(self, p=None) -> Material:
        return self.Shape.MaterialAt(p)


class OBJ:
    """PTSharpCore.OBJ (OBJ.cs), parsed natively by libptsharp_hip.so (pt_obj_load)
    with the reference's quirks; see include/ptsharp_hip.h and DESIGN.md §9a."""

    @staticmethod
    def Load(path: str, parent: "Material" = None) -> Mesh:
        lib = _abi.load_library()
        md = _abi.pt_mesh_data()
        rc = lib.pt_obj_load(str(path).encode(), C.byref(md))
        if rc != 0:
            raise _abi.PTError(rc, "pt_obj_load", lib.pt_obj_last_error().decode())
        try:
            n = md.num_triangles
            arr = lambda p: np.ctypeslib.as_array(p, shape=(n, 3)).copy() if n else np.zeros((0, 3), np.float32)
            m = Mesh(arr(md.v1), arr(md.v2), arr(md.v3), arr(md.n1), arr(md.n2), arr(md.n3),
                     t1=arr(md.t1), t2=arr(md.t2), t3=arr(md.t3))
        finally:
            lib.pt_mesh_free(C.byref(md))
        if parent is not None:
            m.SetMaterial(parent)
        return m


class Scene:
    """PTSharpCore.Scene (Scene.cs).  Shapes keep insertion order; emissive
    shapes are registered as lights exactly as Scene.Add does (Scene.cs:29-38)."""

    def __init__(self):
        self.Shapes: list = []
        self.Lights: list = []
        self.Color = Colour()
        self.Texture = None        # Scene.Texture: environment map (Scene.cs:12, Sampler.cs:177-189)
        self.TextureAngle = 0.0    # Scene.TextureAngle
        self._flat = None

    def Add(self, shape) -> None:
        if isinstance(shape, Mesh):
            shape = shape.copy()  # Mesh is a struct: Scene.Add stores a boxed copy
        self.Shapes.append(shape)
        if shape.MaterialAt().Emittance > 0:
            self.Lights.append(shape)
        self._flat = None

    def AddRange(self, shapes) -> None:
        for s in shapes:
            self.Add(s)

    def Compile(self):
        if self._flat is None:
            self._flat = FlatScene(self)
        return self._flat


class FlatScene:
    """Caller-owned arrays for pt_scene_desc, plus the ctypes struct pointing at them."""

    def __init__(self, scene: Scene):
        mats, mat_ids = [], {}
        texs, tex_ids = [], {}

        def tid(t) -> int:   # 1-based texture slot, 0 = null
            if t is None:
                return 0
            if not isinstance(t, ColorTexture):
                raise _abi.PTError(_abi.PT_ERR_UNSUPPORTED, "Scene.flatten", f"{type(t).__name__} is not on the GPU path")
            if id(t) not in tex_ids:
                texs.append(t)
                tex_ids[id(t)] = len(texs)
            return tex_ids[id(t)]

        def mid(m: Material) -> int:
            k = m.key()
            if k not in mat_ids:
                mat_ids[k] = len(mats)
                mats.append(m)
            return mat_ids[k]

        kinds, idxs = [], []
        sph_c, sph_r, sph_m = [], [], []
        cub_a, cub_b, cub_m = [], [], []
        pl_p, pl_n, pl_m = [], [], []
        tri_parts = []  # list of (v1,v2,v3,n1,n2,n3,mat,t1,t2,t3)
        ntri = 0
        mesh_first, mesh_count = [], []
        sdf_nodes, sdf_children, sdf_ids = [], [], {}
        sdf_shapes, volumes, vol_keep, xforms = [], [], [], []
        inner_meshes = {}

        def sdf_node(n) -> int:   # post-order: children before their parent
            if id(n) in sdf_ids:
                return sdf_ids[id(n)]
            kids = [sdf_node(c) for c in n.children]
            nd = _abi.pt_sdf_node()
            nd.op, nd.num_children, nd.first_child = n.op, len(kids), len(sdf_children)
            sdf_children.extend(kids)
            for k, v in enumerate(n.params):
                nd.params[k] = v
            if n.matrix is not None:
                for k, v in enumerate(n.matrix.m.reshape(-1)):
                    nd.matrix[k] = float(v)
                for k, v in enumerate(n.inverse.m.reshape(-1)):
                    nd.inverse[k] = float(v)
            sdf_ids[id(n)] = len(sdf_nodes)
            sdf_nodes.append(nd)
            return sdf_ids[id(n)]

        def ext(s):
            """(kind, index) of a shape that lives in the per-kind arrays only (inner of a TransformedShape)."""
            if isinstance(s, Sphere):
                sph_c.append(s.Center.f32()); sph_r.append(s.Radius); sph_m.append(mid(s.Material))
                return _abi.SHAPE_SPHERE, len(sph_r) - 1
            if isinstance(s, Cube):
                cub_a.append(s.Min.f32()); cub_b.append(s.Max.f32()); cub_m.append(mid(s.Material))
                return _abi.SHAPE_CUBE, len(cub_m) - 1
            if isinstance(s, Plane):
                pl_p.append(s.Point.f32()); pl_n.append(s.Normal.f32()); pl_m.append(mid(s.Material))
                return _abi.SHAPE_PLANE, len(pl_m) - 1
            if isinstance(s, SDFShape):
                sdf_shapes.append((sdf_node(s.SDF), mid(s.Material)))
                return _abi.SHAPE_SDF, len(sdf_shapes) - 1
            if isinstance(s, Volume):
                wins = (_abi.pt_volume_window * max(1, len(s.Windows)))()
                for k, w in enumerate(s.Windows):
                    wins[k] = _abi.pt_volume_window(w.Lo, w.Hi, mid(w.VolumeWindowMaterial), 0)
                vol_keep.append((s.Data, wins))
                volumes.append(_abi.pt_volume(s.W, s.H, s.D, len(s.Windows), s.ZScale,
                                              s.Data.ctypes.data_as(C.POINTER(C.c_double)),
                                              C.cast(wins, C.POINTER(_abi.pt_volume_window)),
                                              (C.c_float * 3)(*s.Box.Min.f32()), (C.c_float * 3)(*s.Box.Max.f32())))
                return _abi.SHAPE_VOLUME, len(volumes) - 1
            if isinstance(s, Mesh):   # an instanced mesh: its triangles in object space, not in Scene.Shapes
                if id(s) not in inner_meshes:
                    remap = np.array([mid(m) for m in s.materials], np.int32)
                    tri_parts.append((s.v1, s.v2, s.v3, s.n1, s.n2, s.n3, remap[s.mat_index], s.t1, s.t2, s.t3))
                    nonlocal ntri
                    mesh_first.append(ntri); mesh_count.append(len(s))
                    ntri += len(s)
                    inner_meshes[id(s)] = len(mesh_first) - 1
                return _abi.SHAPE_MESH, inner_meshes[id(s)]
            raise _abi.PTError(_abi.PT_ERR_UNSUPPORTED, "Scene.flatten",
                               f"{type(s).__name__} inside a TransformedShape is not on the GPU path")

        for s in scene.Shapes:
            if isinstance(s, Sphere):
                kinds.append(_abi.SHAPE_SPHERE); idxs.append(len(sph_r))
                sph_c.append(s.Center.f32()); sph_r.append(s.Radius); sph_m.append(mid(s.Material))
            elif isinstance(s, Cube):
                kinds.append(_abi.SHAPE_CUBE); idxs.append(len(cub_m))
                cub_a.append(s.Min.f32()); cub_b.append(s.Max.f32()); cub_m.append(mid(s.Material))
            elif isinstance(s, Plane):
                kinds.append(_abi.SHAPE_PLANE); idxs.append(len(pl_m))
                pl_p.append(s.Point.f32()); pl_n.append(s.Normal.f32()); pl_m.append(mid(s.Material))
            elif isinstance(s, Triangle):
                kinds.append(_abi.SHAPE_TRIANGLE); idxs.append(ntri)
                tri_parts.append(tuple(np.array([getattr(s, a).f32()], np.float32)
                                       for a in ("V1", "V2", "V3", "N1", "N2", "N3"))
                                 + (np.array([mid(s.Material)], np.int32),)
                                 + tuple(np.array([getattr(s, a).f32()], np.float32) for a in ("T1", "T2", "T3")))
                ntri += 1
            elif isinstance(s, (SDFShape, Volume)):
                k, i = ext(s)
                kinds.append(k); idxs.append(i)
            elif isinstance(s, TransformedShape):
                k, i = ext(s.Shape)
                x = _abi.pt_transformed_shape()
                x.shape_kind, x.shape_index = k, i
                for j, v in enumerate(s.Matrix.m.reshape(-1)):
                    x.matrix[j] = float(v)
                for j, v in enumerate(s.Inverse.m.reshape(-1)):
                    x.inverse[j] = float(v)
                kinds.append(_abi.SHAPE_TRANSFORMED); idxs.append(len(xforms))
                xforms.append(x)
            elif isinstance(s, Mesh):
                kinds.append(_abi.SHAPE_MESH); idxs.append(len(mesh_first))
                remap = np.array([mid(m) for m in s.materials], np.int32)
                tri_parts.append((s.v1, s.v2, s.v3, s.n1, s.n2, s.n3, remap[s.mat_index], s.t1, s.t2, s.t3))
                mesh_first.append(ntri); mesh_count.append(len(s))
                ntri += len(s)
            else:
                raise _abi.PTError(_abi.PT_ERR_UNSUPPORTED, "Scene.flatten",
                                   f"shape type {type(s).__name__} is not on the GPU path")
        if not mats:
            mid(DEFAULT_MATERIAL)
        self.materials = (_abi.pt_material * len(mats))()
        for i, m in enumerate(mats):
            self.materials[i] = _abi.pt_material((C.c_double * 3)(m.Color.r, m.Color.g, m.Color.b), m.Emittance,
                                                 m.Index, m.Gloss, m.Tint, m.Reflectivity, int(bool(m.Transparent)),
                                                 tid(m.Texture), tid(m.NormalTexture), tid(m.BumpTexture),
                                                 tid(m.GlossTexture), 0, m.BumpMultiplier)
        self.material_list = mats
        arr = lambda T, L: (T * max(1, len(L)))(*L)
        self.sdf_nodes, self.sdf_children = arr(_abi.pt_sdf_node, sdf_nodes), np.array(sdf_children or [0], np.int32)
        self.sdf_shapes = arr(_abi.pt_sdf_shape, [_abi.pt_sdf_shape(r, m) for r, m in sdf_shapes])
        self.volumes, self._vol_keep = arr(_abi.pt_volume, volumes), vol_keep
        self.transformed = arr(_abi.pt_transformed_shape, xforms)
        self.counts_ext = (len(sdf_nodes), len(sdf_shapes), len(volumes), len(xforms))
        self.env_texture = tid(scene.Texture)
        self.env_texture_angle = float(scene.TextureAngle)
        self.texture_list = texs
        self.textures = (_abi.pt_texture * max(1, len(texs)))()
        for i, t in enumerate(texs):
            if t.Width < 2 or t.Height < 2:
                raise _abi.PTError(_abi.PT_ERR_INVALID_ARG, "Scene.flatten", "textures must be at least 2x2")
            self.textures[i] = _abi.pt_texture(t.Width, t.Height, t.Data.ctypes.data_as(C.POINTER(C.c_double)))
        f3 = lambda L: np.ascontiguousarray(np.array(L, np.float32).reshape(-1, 3))
        i32 = lambda L: np.ascontiguousarray(np.array(L, np.int32).reshape(-1))
        self.shape_kind, self.shape_index = i32(kinds), i32(idxs)
        self.sphere_center, self.sphere_radius, self.sphere_material = f3(sph_c), np.array(sph_r, np.float64), i32(sph_m)
        self.cube_min, self.cube_max, self.cube_material = f3(cub_a), f3(cub_b), i32(cub_m)
        self.plane_point, self.plane_normal, self.plane_material = f3(pl_p), f3(pl_n), i32(pl_m)
        if tri_parts:
            cat = [np.ascontiguousarray(np.concatenate([p[k] for p in tri_parts])) for k in range(10)]
        else:
            cat = [np.zeros((0, 3), np.float32)] * 6 + [np.zeros(0, np.int32)] + [np.zeros((0, 3), np.float32)] * 3
        (self.tri_v1, self.tri_v2, self.tri_v3, self.tri_n1, self.tri_n2, self.tri_n3) = cat[:6]
        self.tri_material = cat[6].astype(np.int32)
        self.tri_t1, self.tri_t2, self.tri_t3 = (np.ascontiguousarray(a, np.float32) for a in cat[7:10])
        self.mesh_first, self.mesh_count = i32(mesh_first), i32(mesh_count)
        self.env = scene.Color.tuple()
        self.desc = self._make_desc(_abi.pt_scene_desc)

    def _make_desc(self, cls):
        P = lambda a, t: a.ctypes.data_as(C.POINTER(t)) if a.size else C.POINTER(t)()
        fl, db, it = C.c_float, C.c_double, C.c_int32
        return cls(len(self.material_list), C.cast(self.materials, C.POINTER(_abi.pt_material)),
                   len(self.shape_kind), P(self.shape_kind, it), P(self.shape_index, it),
                   len(self.sphere_radius), P(self.sphere_center, fl), P(self.sphere_radius, db),
                   P(self.sphere_material, it),
                   len(self.cube_material), P(self.cube_min, fl), P(self.cube_max, fl), P(self.cube_material, it),
                   len(self.plane_material), P(self.plane_point, fl), P(self.plane_normal, fl),
                   P(self.plane_material, it),
                   len(self.tri_material), P(self.tri_v1, fl), P(self.tri_v2, fl), P(self.tri_v3, fl),
                   P(self.tri_n1, fl), P(self.tri_n2, fl), P(self.tri_n3, fl), P(self.tri_material, it),
                   len(self.mesh_first), P(self.mesh_first, it), P(self.mesh_count, it),
                   (C.c_double * 3)(*self.env),
                   len(self.texture_list), C.cast(self.textures, C.POINTER(_abi.pt_texture)),
                   P(self.tri_t1, fl), P(self.tri_t2, fl), P(self.tri_t3, fl),
                   self.env_texture, 0, self.env_texture_angle,
                   self.counts_ext[0], C.cast(self.sdf_nodes, C.POINTER(_abi.pt_sdf_node)),
                   self.sdf_children.ctypes.data_as(C.POINTER(C.c_int32)),
                   self.counts_ext[1], C.cast(self.sdf_shapes, C.POINTER(_abi.pt_sdf_shape)),
                   self.counts_ext[2], C.cast(self.volumes, C.POINTER(_abi.pt_volume)),
                   self.counts_ext[3], C.cast(self.transformed, C.POINTER(_abi.pt_transformed_shape)))

    @property
    def num_triangles(self) -> int:
        return len(self.tri_material)


class Camera:
    """PTSharpCore.Camera (Camera.cs): LookAt + SetFocus."""

    def __init__(self):
        self.p = self.u = self.v = self.w = Vector()
        self.m = 0.0
        self.focalDistance = 0.0
        self.apertureRadius = 0.0
        self.fovy = 0.0

    @staticmethod
    def LookAt(eye: Vector, center: Vector, up: Vector, fovy: float) -> "Camera":
        c = Camera()
        c.fovy = fovy
        c.p = eye
        c.w = center.Sub(eye).Normalize()
        c.u = up.Cross(c.w).Normalize()
        c.v = c.w.Cross(c.u).Normalize()
        c.m = 1 / math.tan(fovy * math.pi / 360)
        return c

    def SetFocus(self, focalPoint: Vector, apertureRadius: float) -> None:
        self.focalDistance = focalPoint.Sub(self.p).Length()
        self.apertureRadius = apertureRadius

    def to_c(self, cls=_abi.pt_camera):
        a = lambda v: (C.c_float * 3)(*v.f32())
        return cls(a(self.p), a(self.u), a(self.v), a(self.w), self.m, self.focalDistance, self.apertureRadius)


class DefaultSampler:
    """PTSharpCore.DefaultSampler (Sampler.cs:10-145)."""

    def __init__(self, fh: int, mb: int, dl: bool, ss: bool, lm: LightMode, sm: SpecularMode):
        self.FirstHitSamples, self.MaxBounces = int(fh), int(mb)
        self.DirectLighting, self.SoftShadows = bool(dl), bool(ss)
        self.LightMode, self.SpecularMode = LightMode(lm), SpecularMode(sm)

    @staticmethod
    def NewSampler(firstHitSamples: int, maxBounces: int) -> "DefaultSampler":
        return DefaultSampler(firstHitSamples, maxBounces, True, True, LightMode.LightModeRandom,
                              SpecularMode.SpecularModeNaive)

    def NewDirectSampler(self) -> "DefaultSampler":
        return DefaultSampler(1, 0, True, False, LightMode.LightModeAll, SpecularMode.SpecularModeAll)

    def SetSpecularMode(self, s: SpecularMode) -> None:
        self.SpecularMode = SpecularMode(s)

    def SetLightMode(self, l: LightMode) -> None:
        self.LightMode = LightMode(l)

    def to_c(self, cls=_abi.pt_sampler):
        return cls(self.FirstHitSamples, self.MaxBounces, int(self.DirectLighting), int(self.SoftShadows),
                   int(self.LightMode), int(self.SpecularMode))
