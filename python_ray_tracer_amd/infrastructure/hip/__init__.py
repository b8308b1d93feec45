"""HIP (MI355X, gfx950) backend — drop-in for ``ray_tracer/infrastructure/numpy``.

Reference module -> this module:
  numpy/base.py   NumpyVector3D, NumpyVectorArray3D, NumpyRGBColor, NumpyRenderer, FARAWAY
               -> hip/base.py  HipVector3D, HipVectorArray3D, HipRGBColor, HipRenderer, FARAWAY
  numpy/shape.py  NumpySphere, NumpyTexturedSphere -> hip/shape.py  HipSphere, HipTexturedSphere
  numpy/shader.py Texture, TextureChecker, NumpyShader
               -> hip/shader.py Texture, TextureChecker, ImageTexture, HipShader
"""

from .base import (
    FARAWAY,
    HipCameraRays,
    HipRenderer,
    HipRGBColor,
    HipVector3D,
    HipVectorArray3D,
)
from .shader import HipShader, ImageTexture, Texture, TextureChecker
from .shape import HipSphere, HipTexturedSphere

__all__ = [
    "FARAWAY",
    "HipCameraRays",
    "HipRenderer",
    "HipRGBColor",
    "HipShader",
    "HipSphere",
    "HipTexturedSphere",
    "ImageTexture",
    "HipVector3D",
    "HipVectorArray3D",
    "Texture",
    "TextureChecker",
]
