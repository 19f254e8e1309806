"""ptsharp_amd — MI355X-native render hot path for PTSharp (akav/PTSharp).

Host-side mirror of the reference's render API (Renderer, Scene, IShape kinds,
Material, Camera, DefaultSampler, Buffer) over the C-ABI library
libptsharp_hip.so (include/ptsharp_hip.h), whose gfx950 kernels do the
per-pixel work.  There is no CPU fallback: the product path fails loudly when
the HIP library is missing.
"""
from .geometry import Box, Colour, Matrix, Util, Vector
from .scene import (OBJ, Camera, CapsuleSDF, ColorTexture, Cube, CubeSDF, CylinderSDF, DefaultSampler, DifferenceSDF,
                    IntersectionSDF, LightMode, Material, Mesh, Plane, RepeatSDF, ScaleSDF, Scene, SDFShape, SpecularMode,
                    Sphere, SphereSDF, TorusSDF, TransformedShape, TransformSDF, Triangle, UnionSDF, Volume, VolumeWindow)
from .renderer import Buffer, Channel, Renderer, tiles_for_rank, write_png

__all__ = ["Box", "Colour", "Matrix", "Util", "Vector", "Camera", "ColorTexture", "Cube", "DefaultSampler", "LightMode", "Material",
           "Mesh", "OBJ", "Plane", "Scene", "SpecularMode", "Sphere", "Triangle", "SDFShape", "SphereSDF", "CubeSDF",
           "CylinderSDF", "CapsuleSDF", "TorusSDF", "TransformSDF", "ScaleSDF", "UnionSDF", "DifferenceSDF",
           "IntersectionSDF", "RepeatSDF", "Volume", "VolumeWindow", "TransformedShape", "Buffer", "Channel", "Renderer",
           "tiles_for_rank", "write_png"]
