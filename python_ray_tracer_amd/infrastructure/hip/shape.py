"""``HipSphere`` — drop-in for the reference ``NumpySphere`` (``shape.py:10-54``).

The renderer never calls ``intersect`` per shape (intersection is fused into the render kernel); the
method exists for the ``Shape`` contract (``domain.py:43-46``) and for tests, and runs the
``rtx_sphere_intersect`` kernel (same arithmetic as ``shape.py:28-51``).
"""

from __future__ import annotations

import torch

from python_ray_tracer_amd.domain import Shape

from . import _lib as L
from .base import HipVector3D, _as_vector
from .scene_pack import sphere_geometry


class HipSphere(Shape):
    def __init__(self, center, radius: float, shader) -> None:
        self.center = center  # shape.py:23-26
        self.position = center
        self.radius = radius
        self.shader = shader

    def intersect(self, ray_origin, normalized_ray_direction, device=None) -> torch.Tensor:
        """NumpySphere.intersect (shape.py:28-51) on the GPU: float64 distances, FARAWAY (1e39)
        where the ray misses (a tangent ray, disc == 0, is a miss; an origin inside the sphere
        gives the far root)."""
        lib = L.load()
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        D = _as_vector(normalized_ray_direction).to_tensor(dev)
        if D.dim() == 1:
            D = D.reshape(3, 1)
        n = D.shape[1]
        O = _as_vector(ray_origin).to_tensor(dev, n)
        stride = 0 if O.dim() == 1 else n
        c = self.position
        g = torch.from_numpy(sphere_geometry((float(c.x), float(c.y), float(c.z)), self.radius)).to(dev)
        t = torch.empty(n, dtype=torch.float64, device=dev)
        L.check(lib.rtx_sphere_intersect(g.data_ptr(), O.data_ptr(), stride, D.data_ptr(), n, t.data_ptr(),
                                         L.stream_handle(torch.cuda.current_stream(dev))), "rtx_sphere_intersect")
        return t

    def diffusecolor(self, intersection_point):
        # shape.py:53-54 reads an attribute that is never set; the shader's texture is what renders.
        return self.shader.diffuse_color.get_color(intersection_point)


class HipTexturedSphere(HipSphere):
    """Reference ``NumpyTexturedSphere(center, radius, texture_path)`` (shape.py:57-90): a sphere
    whose diffuse colour is an image mapped by spherical coordinates. The reference passes an RGB
    colour as its shader and cannot render (base.py:110); here the image is an ``ImageTexture`` of
    the sphere's shader: by default ``HipShader(0.0, 0.0, 0.5, 0.0, 1.0, ImageTexture(path))`` (pure
    diffuse), or ``shader`` with its ``diffuse_color`` replaced by the image."""

    def __init__(self, center, radius: float, texture_path, shader=None) -> None:
        from .shader import HipShader, ImageTexture

        tex = ImageTexture(texture_path)
        if shader is None:
            shader = HipShader(0.0, 0.0, 0.5, 0.0, 1.0, tex)
        else:
            shader.diffuse_color = tex
        super().__init__(center, radius, shader)
        self.image = tex


__all__ = ["HipSphere", "HipTexturedSphere", "HipVector3D"]
