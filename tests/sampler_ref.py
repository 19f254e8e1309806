"""A second, independent restatement of the reference's bounce and light sampling, written
line by line from the C# in Python (test infrastructure, like tests/obj_ref.py), to pin the
oracle's C++ (oracle/pt_oracle.cpp) where no C# can run:

  Vector.RandomUnitVector / Reflect / Refract / Reflectance   Vector.cs:339-347, 497-536
  Util.Cone                                                   Util.cs:17-32
  Ray.WeightedBounce / ConeBounce / Bounce                    Ray.cs:28-85
  Box.Center / OuterRadius                                    Box.cs:50-52
  Sampler.sampleLight (Sphere, Cylinder, bounding-box light)  Sampler.cs:212-296
  Sampler.sampleLights (LightModeAll / LightModeRandom)       Sampler.cs:191-210

Vector is System.Numerics.Vector3 behind double accessors: fp32 storage, every Add / Sub /
Cross / Normalize / Dot in fp32, MulScalar(double) = float(double(x)·s).  Scalars are fp64
(Python floats; math.sin/cos/acos/asin/tan/sqrt are the platform libm, as std:: is for the
oracle).  Random.Shared is replaced by the counter-based stream of DESIGN.md §3 (draw(key, dim)),
restated here from its definition, not imported.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
EPS = 1e-9                              # Util.EPS (Util.cs:11)
M64 = (1 << 64) - 1
D_REFLECT, D_RUV_Z, D_RUV_A, D_LIGHT, D_SS_RUV_Z, D_SS_RUV_A, D_SS_XY = 2, 3, 4, 5, 6, 7, 8


# ------------------------------------------------------------------ counter-based RNG
def mix64(x: int) -> int:
    x &= M64
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M64
    x ^= x >> 31
    return x


def draw(key: int, dim: int) -> float:
    return float(mix64(key + (dim + 1) * 0x9E3779B97F4A7C15) >> 11) * (1.0 / 9007199254740992.0)


def light_key(key: int, i: int) -> int:
    return mix64(key ^ ((i + 0xBE5466CF34E90C6C) & M64))


# ------------------------------------------------------------------ Vector (fp32 storage)
class Vec:
    __slots__ = ("x", "y", "z")

    def __init__(self, x=0.0, y=0.0, z=0.0):   # new Vector(double, double, double): stored as float
        self.x, self.y, self.z = F32(x), F32(y), F32(z)

    def t(self):
        return (float(self.x), float(self.y), float(self.z))

    def Add(self, b):
        return Vec(self.x + b.x, self.y + b.y, self.z + b.z)

    def Sub(self, b):
        return Vec(self.x - b.x, self.y - b.y, self.z - b.z)

    def Mul(self, b):
        return Vec(self.x * b.x, self.y * b.y, self.z * b.z)

    def MulScalar(self, s: float):
        return Vec(float(self.x) * s, float(self.y) * s, float(self.z) * s)

    def Dot(self, b) -> float:   # Vector3.Dot in fp32, returned as double
        return float((self.x * b.x + self.y * b.y) + self.z * b.z)

    def Cross(self, b):
        return Vec(self.y * b.z - self.z * b.y, self.z * b.x - self.x * b.z, self.x * b.y - self.y * b.x)

    def Length(self) -> float:
        return float(np.sqrt((self.x * self.x + self.y * self.y) + self.z * self.z))

    def Normalize(self):
        ln = np.sqrt((self.x * self.x + self.y * self.y) + self.z * self.z)
        return Vec(self.x / ln, self.y / ln, self.z / ln)

    # Vector.Reflect / Refract / Reflectance with `this` = the normal (Vector.cs:497-536)
    def Reflect(self, i):
        return i.Sub(self.MulScalar(2 * self.Dot(i)))

    def Refract(self, i, n1: float, n2: float):
        nr = n1 / n2
        cosI = -self.Dot(i)
        sinT2 = nr * nr * (1 - cosI * cosI)
        if sinT2 > 1:
            return Vec()
        cosT = math.sqrt(1 - sinT2)
        return i.MulScalar(nr).Add(self.MulScalar(nr * cosI - cosT))

    def Reflectance(self, i, n1: float, n2: float) -> float:
        nr2 = (n1 * n1) / (n2 * n2)
        cosI = -self.Dot(i)
        sinT2 = nr2 * (1 - cosI * cosI)
        if sinT2 > 1:
            return 1.0
        cosT = math.sqrt(1 - sinT2)
        cosI_n1 = n1 * cosI
        cosT_n2 = n2 * cosT
        rOrth = (cosI_n1 - cosT_n2) / (cosI_n1 + cosT_n2)
        rPar = (cosT_n2 - cosI_n1) / (cosT_n2 + cosI_n1)
        return (rOrth * rOrth + rPar * rPar) / 2


def random_unit_vector(key: int, dz: int, da: int) -> Vec:
    """Vector.RandomUnitVector (Vector.cs:339-347): z, a, r, x = Sin(a), y = Cos(a)."""
    z = draw(key, dz) * 2.0 - 1.0
    a = draw(key, da) * 2.0 * math.pi
    r = math.sqrt(1.0 - z * z)
    x = math.sin(a)
    y = math.cos(a)
    return Vec(r * x, r * y, z)


def cone(direction: Vec, theta: float, u: float, v: float, key: int) -> Vec:
    """Util.Cone (Util.cs:17-32); s = direction x q is NOT normalised in the reference."""
    if theta < EPS:
        return direction
    theta = theta * (1 - (2 * math.acos(u) / math.pi))
    m1 = math.sin(theta)
    m2 = math.cos(theta)
    a = v * 2 * math.pi
    q = random_unit_vector(key, D_RUV_Z, D_RUV_A)
    s = direction.Cross(q)
    t = direction.Cross(s)
    return Vec().Add(s.MulScalar(m1 * math.cos(a))).Add(t.MulScalar(m1 * math.sin(a))).Add(direction.MulScalar(m2)).Normalize()


def weighted_bounce(origin: Vec, normal: Vec, u: float, v: float, key: int):
    """Ray.WeightedBounce (Ray.cs:28-35) on the normal ray."""
    radius = math.sqrt(u)
    theta = 2 * math.pi * v
    s = normal.Cross(random_unit_vector(key, D_RUV_Z, D_RUV_A)).Normalize()
    t = normal.Cross(s)
    d = Vec().Add(s.MulScalar(radius * math.cos(theta))).Add(t.MulScalar(radius * math.sin(theta))).Add(
        normal.MulScalar(math.sqrt(1 - u)))
    return origin, d


def bounce(in_dir: Vec, pos: Vec, normal: Vec, inside: bool, material, u: float, v: float, btype: int, key: int):
    """Ray.Bounce (Ray.cs:44-85): returns (origin, direction, reflected, p).
    btype 0 Any, 1 Diffuse, 2 Specular (BounceType.cs); material has Index, Reflectivity, Transparent, Gloss."""
    n1, n2 = 1.0, float(material.Index)
    if inside:
        n1, n2 = n2, n1
    p = float(material.Reflectivity) if material.Reflectivity >= 0 else normal.Reflectance(in_dir, n1, n2)
    if btype == 0:
        reflect = draw(key, D_REFLECT) < p
    else:
        reflect = btype == 2
    if reflect:
        d = normal.Reflect(in_dir)
        return pos, cone(d, float(material.Gloss), u, v, key), True, p
    if material.Transparent:
        rd = normal.Refract(in_dir, n1, n2)
        o = pos.Add(rd.MulScalar(1e-4))
        return o, cone(rd, float(material.Gloss), u, v, key), True, 1 - p
    o, d = weighted_bounce(pos, normal, u, v, key)
    return o, d, False, 1 - p


# ------------------------------------------------------------------ lights
def box_center(mn: Vec, mx: Vec) -> Vec:
    """Box.Center = Anchor((0.5, 0.5, 0.5)) = Min + Size·anchor (Box.cs:44-50)."""
    return mn.Add(mx.Sub(mn).Mul(Vec(0.5, 0.5, 0.5)))


def box_outer_radius(mn: Vec, mx: Vec) -> float:
    return mn.Sub(box_center(mn, mx)).Length()   # Box.cs:52


def net_min(a: float, b: float) -> float:
    """.NET Math.Min(double, double): NaN propagates."""
    if a != a or b != b:
        return float("nan")
    return a if a < b else b


class Light:
    """A Scene.Lights entry: kind 'sphere' (center, radius), 'cylinder' (radius, z0, z1) or 'box'
    (mn, mx: light.BoundingBox()); `identity(kind, index)` answers `hit.Shape == light`;
    colour and emittance are Material.MaterialAt(light, point) (untextured here)."""

    def __init__(self, kind, colour, emittance, identity, center=None, radius=None, mn=None, mx=None, z0=None, z1=None):
        self.kind, self.colour, self.emittance, self.identity = kind, colour, emittance, identity
        self.center, self.radius, self.mn, self.mx, self.z0, self.z1 = center, radius, mn, mx, z0, z1


def sample_light(intersect, n_origin: Vec, n_dir: Vec, light: Light, key: int, soft_shadows: bool = True):
    """Sampler.sampleLight (Sampler.cs:212-296).  intersect(origin, dir) -> (t, kind, index) is
    Scene.Intersect.  Returns (colour (r, g, b), Scene.Intersect calls made)."""
    if light.kind == "sphere":                         # case Sphere sphere:
        radius = float(light.radius)
        center = light.center
    elif light.kind == "cylinder":                     # case Cylinder cylinder:
        radius = float(light.radius)
        center = Vec(0, 0, (light.z0 + light.z1) / 2)
    else:                                              # default: light.BoundingBox()
        radius = box_outer_radius(light.mn, light.mx)
        center = box_center(light.mn, light.mx)
    point = center
    if soft_shadows:
        for k in range(256):   # while (true): the stream's 256 tries stand in for the unbounded loop
            x = draw(key, D_SS_XY + 2 * k) * 2 - 1
            y = draw(key, D_SS_XY + 2 * k + 1) * 2 - 1
            if x * x + y * y <= 1:
                l = center.Sub(n_origin).Normalize()
                u = l.Cross(random_unit_vector(key, D_SS_RUV_Z, D_SS_RUV_A)).Normalize()
                v = l.Cross(u)
                point = center.Add(u.MulScalar(x * radius)).Add(v.MulScalar(y * radius))
                break
    ray_dir = point.Sub(n_origin).Normalize()
    diffuse = ray_dir.Dot(n_dir)
    if diffuse <= 0:
        return (0.0, 0.0, 0.0), 0
    t, hk, hi = intersect(n_origin, ray_dir)
    if not (t < 1e9) or not light.identity(hk, hi):   # !hit.Ok || hit.Shape != light
        return (0.0, 0.0, 0.0), 1
    if light.kind == "cylinder":
        coverage = 1.0
    else:
        hyp = center.Sub(n_origin).Length()
        theta = math.asin(radius / hyp)
        adj = radius / math.tan(theta)
        d = math.cos(theta) * adj
        r = math.sin(theta) * adj
        coverage = (r * r) / (d * d)
        if hyp < radius:
            coverage = 1.0
        coverage = net_min(coverage, 1)
    m = light.emittance * diffuse * coverage
    return tuple(c * m for c in light.colour), 1


def sample_lights(intersect, n_origin: Vec, n_dir: Vec, lights: list, key: int, light_mode: int,
                  soft_shadows: bool = True):
    """Sampler.sampleLights (Sampler.cs:191-210); light_mode 1 = LightModeAll.  The random light
    index is floor(draw·n) (for Random.Next(nLights))."""
    n = len(lights)
    if n == 0:
        return (0.0, 0.0, 0.0), 0
    if light_mode == 1:
        res, rays = (0.0, 0.0, 0.0), 0
        for i, L in enumerate(lights):
            c, r = sample_light(intersect, n_origin, n_dir, L, light_key(key, i), soft_shadows)
            res = (res[0] + c[0], res[1] + c[1], res[2] + c[2])
            rays += r
        return (res[0] / n, res[1] / n, res[2] / n), rays
    idx = min(int(draw(key, D_LIGHT) * n), n - 1)
    c, r = sample_light(intersect, n_origin, n_dir, lights[idx], key, soft_shadows)
    return (c[0] * float(n), c[1] * float(n), c[2] * float(n)), r
