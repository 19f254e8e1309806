"""ptsharp_amd — MI355X-native render hot path for PTSharp (akav/PTSharp).

Host-side mirror of the reference's render API (Renderer, Scene, IShape kinds,
Material, Camera, DefaultSampler, Buffer) over the C-ABI library
libptsharp_hip.so (include/ptsharp_hip.h), whose gfx950 kernels do the
per-pixel work.  There is no CPU fallback: the product path fails loudly when
the HIP library is missing.
"""
from .geometry import Box, Colour, Matrix, Util, Vector
from .scene import (OBJ, Camera, ColorTexture, Cube, DefaultSampler, LightMode, Material, Mesh, Plane, Scene, SpecularMode,
                    Sphere, Triangle)
from .renderer import Buffer, Channel, Renderer, tiles_for_rank, write_png

__all__ = ["Box", "Colour", "Matrix", "Util", "Vector", "Camera", "ColorTexture", "Cube", "DefaultSampler", "LightMode", "Material",
           "Mesh", "OBJ", "Plane", "Scene", "SpecularMode", "Sphere", "Triangle", "Buffer", "Channel", "Renderer",
           "tiles_for_rank", "write_png"]
