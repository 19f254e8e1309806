"""Host-side mirror of PTSharp's numeric types: Vector (fp32 storage, fp64 API),
Colour (fp64), Box, Matrix and Util (PTSharpCore/Vector.cs:193-543,
Colour.cs, Box.cs, Matrix.cs, Util.cs).

These run once per scene build, not per ray; they reproduce the reference's
rounding (every Vector op re-rounds to fp32, MulScalar(double) = float(x*s))
so the flattened scene handed to the GPU is the one the C# side would build.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32
F64 = np.float64

_ERR = np.seterr  # keep a handle; ops below run under errstate(all="ignore")


def _f(x) -> np.float32:
    return np.float32(x)


class Vector:
    """PTSharpCore.Vector: a System.Numerics.Vector3 behind double accessors."""

    __slots__ = ("_x", "_y", "_z")

    def __init__(self, x=0.0, y=0.0, z=0.0):
        with np.errstate(all="ignore"):
            self._x = np.float32(x)
            self._y = np.float32(y)
            self._z = np.float32(z)

    # accessors return double, as Vector.X/Y/Z do
    @property
    def X(self) -> float:
        return float(self._x)

    @property
    def Y(self) -> float:
        return float(self._y)

    @property
    def Z(self) -> float:
        return float(self._z)

    def f32(self) -> tuple:
        return (self._x, self._y, self._z)

    def __iter__(self):
        return iter((self.X, self.Y, self.Z))

    def __repr__(self):
        return f"({self.X}, {self.Y}, {self.Z})"

    def __eq__(self, o):
        return isinstance(o, Vector) and self.X == o.X and self.Y == o.Y and self.Z == o.Z

    def __hash__(self):
        return hash((self.X, self.Y, self.Z))

    @staticmethod
    def _mk32(x, y, z) -> "Vector":
        v = Vector.__new__(Vector)
        v._x, v._y, v._z = x, y, z
        return v

    def Add(self, b):
        with np.errstate(all="ignore"):
            return Vector._mk32(self._x + b._x, self._y + b._y, self._z + b._z)

    def Sub(self, b):
        with np.errstate(all="ignore"):
            return Vector._mk32(self._x - b._x, self._y - b._y, self._z - b._z)

    def Mul(self, b):
        with np.errstate(all="ignore"):
            return Vector._mk32(self._x * b._x, self._y * b._y, self._z * b._z)

    def Div(self, b):
        with np.errstate(all="ignore"):
            return Vector._mk32(self._x / b._x, self._y / b._y, self._z / b._z)

    def MulScalar(self, s: float):
        with np.errstate(all="ignore"):
            return Vector(F64(self._x) * s, F64(self._y) * s, F64(self._z) * s)

    def DivScalar(self, s: float):
        with np.errstate(all="ignore"):
            return Vector(F64(self._x) / s, F64(self._y) / s, F64(self._z) / s)

    def Dot(self, b) -> float:
        with np.errstate(all="ignore"):
            s = (self._x * b._x + self._y * b._y)
            return float(s + self._z * b._z)

    def Cross(self, b):
        with np.errstate(all="ignore"):
            return Vector._mk32(self._y * b._z - self._z * b._y, self._z * b._x - self._x * b._z,
                                self._x * b._y - self._y * b._x)

    def Length(self) -> float:
        with np.errstate(all="ignore"):
            return float(np.sqrt(np.float32(self.Dot(self))))

    def Normalize(self):
        with np.errstate(all="ignore"):
            l = np.sqrt(np.float32(self.Dot(self)))
            return Vector._mk32(self._x / l, self._y / l, self._z / l)

    def Negate(self):
        return Vector._mk32(-self._x, -self._y, -self._z)

    def Min(self, b):
        return Vector(net_min(self.X, b.X), net_min(self.Y, b.Y), net_min(self.Z, b.Z))

    def Max(self, b):
        return Vector(net_max(self.X, b.X), net_max(self.Y, b.Y), net_max(self.Z, b.Z))

    def MinComponent(self) -> float:
        return net_min(net_min(self.X, self.Y), self.Z)

    def MaxComponent(self) -> float:
        return net_max(net_max(self.X, self.Y), self.Z)


def net_max(a: float, b: float) -> float:
    """System.Math.Max(double, double)."""
    if a != b:
        if not math.isnan(a):
            return a if b < a else b
        return a
    return a if math.copysign(1.0, b) < 0 else b


def net_min(a: float, b: float) -> float:
    """System.Math.Min(double, double)."""
    if a != b:
        if not math.isnan(a):
            return a if a < b else b
        return a
    return a if math.copysign(1.0, a) < 0 else b


class Colour:
    """PTSharpCore.Colour (fp64 r, g, b)."""

    __slots__ = ("r", "g", "b")

    def __init__(self, r=0.0, g=0.0, b=0.0):
        self.r, self.g, self.b = float(r), float(g), float(b)

    def __repr__(self):
        return f"Colour({self.r}, {self.g}, {self.b})"

    def __eq__(self, o):
        return isinstance(o, Colour) and (self.r, self.g, self.b) == (o.r, o.g, o.b)

    def tuple(self):
        return (self.r, self.g, self.b)

    @staticmethod
    def HexColor(x: int) -> "Colour":
        # Colour.HexColor (Colour.cs:125-132): float division, then Pow(2.2f)
        red = float(np.float32(((x >> 16) & 0xFF) / np.float32(255.0)))
        green = float(np.float32(((x >> 8) & 0xFF) / np.float32(255.0)))
        blue = float(np.float32((x & 0xFF) / np.float32(255.0)))
        return Colour(red, green, blue).Pow(float(np.float32(2.2)))

    def Pow(self, b: float) -> "Colour":
        return Colour(math.pow(self.r, b), math.pow(self.g, b), math.pow(self.b, b))

    def MulScalar(self, s):
        return Colour(self.r * s, self.g * s, self.b * s)

    def Add(self, o):
        return Colour(self.r + o.r, self.g + o.g, self.b + o.b)

    def Mul(self, o):
        return Colour(self.r * o.r, self.g * o.g, self.b * o.b)

    def DivScalar(self, s):
        return Colour(self.r / s, self.g / s, self.b / s)


Colour.Black = Colour(0, 0, 0)
Colour.White = Colour(1, 1, 1)


class Box:
    """PTSharpCore.Box (Box.cs)."""

    def __init__(self, mn: Vector = None, mx: Vector = None):
        self.Min = mn if mn is not None else Vector()
        self.Max = mx if mx is not None else Vector()

    def Size(self) -> Vector:
        return self.Max.Sub(self.Min)

    def Anchor(self, anchor: Vector) -> Vector:
        return self.Min.Add(self.Size().Mul(anchor))

    def Center(self) -> Vector:
        return self.Anchor(Vector(0.5, 0.5, 0.5))

    def OuterRadius(self) -> float:
        return self.Min.Sub(self.Center()).Length()

    def Extend(self, b: "Box") -> "Box":
        return Box(self.Min.Min(b.Min), self.Max.Max(b.Max))


class Matrix:
    """PTSharpCore.Matrix (Matrix.cs): 4x4 fp64, row-major M11..M44."""

    def __init__(self, m=None):
        self.m = np.array(m, dtype=np.float64).reshape(4, 4) if m is not None else np.zeros((4, 4))

    @staticmethod
    def Identity() -> "Matrix":
        return Matrix(np.eye(4))

    @staticmethod
    def TranslateM(v: Vector) -> "Matrix":
        # Matrix.Translate ignores `this` (Matrix.cs:33-36)
        return Matrix([[1, 0, 0, v.X], [0, 1, 0, v.Y], [0, 0, 1, v.Z], [0, 0, 0, 1]])

    @staticmethod
    def ScaleM(v: Vector) -> "Matrix":
        return Matrix([[v.X, 0, 0, 0], [0, v.Y, 0, 0], [0, 0, v.Z, 0], [0, 0, 0, 1]])

    @staticmethod
    def RotateM(v: Vector, a: float) -> "Matrix":
        # Matrix.Rotate (Matrix.cs:43-53)
        v = v.Normalize()
        x, y, z = v.X, v.Y, v.Z
        s, c = math.sin(a), math.cos(a)
        m = 1 - c
        return Matrix([[m * x * x + c, m * x * y + z * s, m * z * x - y * s, 0],
                       [m * x * y - z * s, m * y * y + c, m * y * z + x * s, 0],
                       [m * z * x + y * s, m * y * z - x * s, m * z * z + c, 0],
                       [0, 0, 0, 1]])

    def Mul(self, b: "Matrix") -> "Matrix":
        # Matrix.Mul (Matrix.cs:111-131): explicit left-to-right sums
        a, bb = self.m, b.m
        out = np.empty((4, 4))
        for i in range(4):
            for j in range(4):
                out[i, j] = a[i, 0] * bb[0, j] + a[i, 1] * bb[1, j] + a[i, 2] * bb[2, j] + a[i, 3] * bb[3, j]
        return Matrix(out)

    def Determinant(self) -> float:
        """Matrix.Determinant (Matrix.cs:179-193), the reference's term order."""
        a = [[float(x) for x in row] for row in self.m]
        return (a[0][0] * a[1][1] * a[2][2] * a[3][3] - a[0][0] * a[1][1] * a[2][3] * a[3][2]
            + a[0][0] * a[1][2] * a[2][3] * a[3][1] - a[0][0] * a[1][2] * a[2][1] * a[3][3]
            + a[0][0] * a[1][3] * a[2][1] * a[3][2] - a[0][0] * a[1][3] * a[2][2] * a[3][1]
            - a[0][1] * a[1][2] * a[2][3] * a[3][0] + a[0][1] * a[1][2] * a[2][0] * a[3][3]
            - a[0][1] * a[1][3] * a[2][0] * a[3][2] + a[0][1] * a[1][3] * a[2][2] * a[3][0]
            - a[0][1] * a[1][0] * a[2][2] * a[3][3] + a[0][1] * a[1][0] * a[2][3] * a[3][2]
            + a[0][2] * a[1][3] * a[2][0] * a[3][1] - a[0][2] * a[1][3] * a[2][1] * a[3][0]
            + a[0][2] * a[1][0] * a[2][1] * a[3][3] - a[0][2] * a[1][0] * a[2][3] * a[3][1]
            + a[0][2] * a[1][1] * a[2][3] * a[3][0] - a[0][2] * a[1][1] * a[2][0] * a[3][3]
            - a[0][3] * a[1][0] * a[2][1] * a[3][2] + a[0][3] * a[1][0] * a[2][2] * a[3][1]
            - a[0][3] * a[1][1] * a[2][2] * a[3][0] + a[0][3] * a[1][1] * a[2][0] * a[3][2]
            - a[0][3] * a[1][2] * a[2][0] * a[3][1] + a[0][3] * a[1][2] * a[2][1] * a[3][0])

    def Inverse(self) -> "Matrix":
        """Matrix.Inverse (Matrix.cs:196-216), the reference's cofactor sums in order."""
        a = [[float(x) for x in row] for row in self.m]
        d = self.Determinant()
        o = np.zeros((4, 4))
        o[0, 0] = (a[1][2] * a[2][3] * a[3][1] - a[1][3] * a[2][2] * a[3][1] + a[1][3] * a[2][1] * a[3][2]
            - a[1][1] * a[2][3] * a[3][2] - a[1][2] * a[2][1] * a[3][3] + a[1][1] * a[2][2] * a[3][3]) / d
        o[0, 1] = (a[0][3] * a[2][2] * a[3][1] - a[0][2] * a[2][3] * a[3][1] - a[0][3] * a[2][1] * a[3][2]
            + a[0][1] * a[2][3] * a[3][2] + a[0][2] * a[2][1] * a[3][3] - a[0][1] * a[2][2] * a[3][3]) / d
        o[0, 2] = (a[0][2] * a[1][3] * a[3][1] - a[0][3] * a[1][2] * a[3][1] + a[0][3] * a[1][1] * a[3][2]
            - a[0][1] * a[1][3] * a[3][2] - a[0][2] * a[1][1] * a[3][3] + a[0][1] * a[1][2] * a[3][3]) / d
        o[0, 3] = (a[0][3] * a[1][2] * a[2][1] - a[0][2] * a[1][3] * a[2][1] - a[0][3] * a[1][1] * a[2][2]
            + a[0][1] * a[1][3] * a[2][2] + a[0][2] * a[1][1] * a[2][3] - a[0][1] * a[1][2] * a[2][3]) / d
        o[1, 0] = (a[1][3] * a[2][2] * a[3][0] - a[1][2] * a[2][3] * a[3][0] - a[1][3] * a[2][0] * a[3][2]
            + a[1][0] * a[2][3] * a[3][2] + a[1][2] * a[2][0] * a[3][3] - a[1][0] * a[2][2] * a[3][3]) / d
        o[1, 1] = (a[0][2] * a[2][3] * a[3][0] - a[0][3] * a[2][2] * a[3][0] + a[0][3] * a[2][0] * a[3][2]
            - a[0][0] * a[2][3] * a[3][2] - a[0][2] * a[2][0] * a[3][3] + a[0][0] * a[2][2] * a[3][3]) / d
        o[1, 2] = (a[0][3] * a[1][2] * a[3][0] - a[0][2] * a[1][3] * a[3][0] - a[0][3] * a[1][0] * a[3][2]
            + a[0][0] * a[1][3] * a[3][2] + a[0][2] * a[1][0] * a[3][3] - a[0][0] * a[1][2] * a[3][3]) / d
        o[1, 3] = (a[0][2] * a[1][3] * a[2][0] - a[0][3] * a[1][2] * a[2][0] + a[0][3] * a[1][0] * a[2][2]
            - a[0][0] * a[1][3] * a[2][2] - a[0][2] * a[1][0] * a[2][3] + a[0][0] * a[1][2] * a[2][3]) / d
        o[2, 0] = (a[1][1] * a[2][3] * a[3][0] - a[1][3] * a[2][1] * a[3][0] + a[1][3] * a[2][0] * a[3][1]
            - a[1][0] * a[2][3] * a[3][1] - a[1][1] * a[2][0] * a[3][3] + a[1][0] * a[2][1] * a[3][3]) / d
        o[2, 1] = (a[0][3] * a[2][1] * a[3][0] - a[0][1] * a[2][3] * a[3][0] - a[0][3] * a[2][0] * a[3][1]
            + a[0][0] * a[2][3] * a[3][1] + a[0][1] * a[2][0] * a[3][3] - a[0][0] * a[2][1] * a[3][3]) / d
        o[2, 2] = (a[0][1] * a[1][3] * a[3][0] - a[0][3] * a[1][1] * a[3][0] + a[0][3] * a[1][0] * a[3][1]
            - a[0][0] * a[1][3] * a[3][1] - a[0][1] * a[1][0] * a[3][3] + a[0][0] * a[1][1] * a[3][3]) / d
        o[2, 3] = (a[0][3] * a[1][1] * a[2][0] - a[0][1] * a[1][3] * a[2][0] - a[0][3] * a[1][0] * a[2][1]
            + a[0][0] * a[1][3] * a[2][1] + a[0][1] * a[1][0] * a[2][3] - a[0][0] * a[1][1] * a[2][3]) / d
        o[3, 0] = (a[1][2] * a[2][1] * a[3][0] - a[1][1] * a[2][2] * a[3][0] - a[1][2] * a[2][0] * a[3][1]
            + a[1][0] * a[2][2] * a[3][1] + a[1][1] * a[2][0] * a[3][2] - a[1][0] * a[2][1] * a[3][2]) / d
        o[3, 1] = (a[0][1] * a[2][2] * a[3][0] - a[0][2] * a[2][1] * a[3][0] + a[0][2] * a[2][0] * a[3][1]
            - a[0][0] * a[2][2] * a[3][1] - a[0][1] * a[2][0] * a[3][2] + a[0][0] * a[2][1] * a[3][2]) / d
        o[3, 2] = (a[0][2] * a[1][1] * a[3][0] - a[0][1] * a[1][2] * a[3][0] - a[0][2] * a[1][0] * a[3][1]
            + a[0][0] * a[1][2] * a[3][1] + a[0][1] * a[1][0] * a[3][2] - a[0][0] * a[1][1] * a[3][2]) / d
        o[3, 3] = (a[0][1] * a[1][2] * a[2][0] - a[0][2] * a[1][1] * a[2][0] + a[0][2] * a[1][0] * a[2][1]
            - a[0][0] * a[1][2] * a[2][1] - a[0][1] * a[1][0] * a[2][2] + a[0][0] * a[1][1] * a[2][2]) / d
        return Matrix(o)

    def Transpose(self) -> "Matrix":   # Matrix.cs:176
        return Matrix(self.m.T.copy())

    def MulPosition(self, b: Vector) -> Vector:
        """Matrix.MulPosition (Matrix.cs:134-141)."""
        m = self.m
        return Vector(*[((m[r, 0] * b.X + m[r, 1] * b.Y) + m[r, 2] * b.Z) + m[r, 3] for r in range(3)])

    def MulBox(self, box: "Box") -> "Box":
        """Matrix.MulBox (Matrix.cs:156-173)."""
        m = self.m
        r, u, b, t = (Vector(m[0, k], m[1, k], m[2, k]) for k in range(4))
        xa, xb = r.MulScalar(box.Min.X), r.MulScalar(box.Max.X)
        ya, yb = u.MulScalar(box.Min.Y), u.MulScalar(box.Max.Y)
        za, zb = b.MulScalar(box.Min.Z), b.MulScalar(box.Max.Z)
        xa, xb = xa.Min(xb), xa.Max(xb)
        ya, yb = ya.Min(yb), ya.Max(yb)
        za, zb = za.Min(zb), za.Max(zb)
        return Box(xa.Add(ya).Add(za).Add(t), xb.Add(yb).Add(zb).Add(t))

    def MulPosition_arrays(self, p: np.ndarray) -> np.ndarray:
        """MulPosition on an [n,3] float32 array (Matrix.cs:134-141)."""
        m = self.m
        x, y, z = (p[:, k].astype(np.float64) for k in range(3))
        out = np.empty_like(p, dtype=np.float32)
        for r in range(3):
            out[:, r] = (((m[r, 0] * x + m[r, 1] * y) + m[r, 2] * z) + m[r, 3]).astype(np.float32)
        return out

    def MulDirection_arrays(self, d: np.ndarray) -> np.ndarray:
        """MulDirection on an [n,3] float32 array: fp64 product → fp32 → Normalize (Matrix.cs:144-150)."""
        m = self.m
        x, y, z = (d[:, k].astype(np.float64) for k in range(3))
        out = np.empty_like(d, dtype=np.float32)
        for r in range(3):
            out[:, r] = ((m[r, 0] * x + m[r, 1] * y) + m[r, 2] * z).astype(np.float32)
        return normalize_rows(out)


def dot_rows(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Vector3.Dot on float32 rows: (x*x' + y*y') + z*z' in fp32."""
    with np.errstate(all="ignore"):
        return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]


def normalize_rows(a: np.ndarray) -> np.ndarray:
    """Vector3.Normalize on float32 rows: v / sqrt(dot(v, v)) in fp32."""
    a = np.asarray(a, dtype=np.float32)
    with np.errstate(all="ignore"):
        l = np.sqrt(dot_rows(a, a)).astype(np.float32)
        return (a / l[:, None]).astype(np.float32)


def cross_rows(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    with np.errstate(all="ignore"):
        return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                         a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], axis=1).astype(np.float32)


class Util:
    INF = 1e9
    EPS = 1e-9

    @staticmethod
    def Radians(degrees: float) -> float:
        return degrees * math.pi / 180

    @staticmethod
    def Degrees(radians: float) -> float:
        return radians * 180 / math.pi
