"""Scene description types — the input data model of the render path.

Mirrors the reference's domain layer (`/root/reference/ray_tracer/domain.py:5-59`) name for name
so a scene written against the reference reads the same here:

* ``Vector3D`` / ``RGBColor``     — ``domain.py:5-11``
* ``Camera``                      — ``domain.py:14-23`` (position, width, height)
* ``PointLight``                  — ``domain.py:26-30``
* ``DomeLight``                   — ``domain.py:33-40``
* ``Shape`` (ABC)                 — ``domain.py:43-50``
* ``Scene3D``                     — ``domain.py:53-59``

These are plain host-side containers. The HIP backend flattens them into one float64 blob per
scene (see ``infrastructure/hip/scene_pack.py``); nothing here touches the GPU.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass


class Vector3D:
    """Three components, scalars or arrays (reference ``domain.py:5-7``)."""

    def __init__(self, x, y, z) -> None:
        (self.x, self.y, self.z) = (x, y, z)

    def components(self) -> tuple:
        return (self.x, self.y, self.z)

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.x!r}, {self.y!r}, {self.z!r})"


class RGBColor(Vector3D):
    """Reference ``domain.py:10-11``."""


@dataclass
class Camera:
    """Observation point; the screen is fixed at world z=0 (reference ``domain.py:14-23``,
    screen construction in ``infrastructure/numpy/base.py:123-141``)."""

    position: Vector3D
    width: int
    height: int


@dataclass
class PointLight:
    """Reference ``domain.py:26-30``. Only ``scene.lights[0]`` is ever used as the point light
    (``shader.py:75``)."""

    position: Vector3D


@dataclass
class DomeLight:
    """Sky light (reference ``domain.py:33-40``); every DomeLight in ``scene.lights`` adds its
    intensity, the colour of the last one wins (``shader.py:234-244``)."""

    intensity: float
    color: RGBColor


class Shape(ABC):
    """Reference ``domain.py:43-50``."""

    @abstractmethod
    def intersect(self, ray_origin, normalized_ray_direction):
        pass

    @abstractmethod
    def diffusecolor(self, intersection_point):
        pass


@dataclass
class Scene3D:
    """Reference ``domain.py:53-59``."""

    shapes: list
    lights: list
    camera: Camera
