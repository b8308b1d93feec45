"""Scene specifications used by the benchmarks, the tests and the golden-fixture generator.

A *scene spec* is a plain JSON-able dict, so the same scene can be instantiated with this
package's classes (``build_scene``), with the reference's classes (the fixture generator under
``tests/golden/``) and by the CPU oracle (``oracle/numpy_oracle.py``) without any of them
importing each other.

Scenes:

* ``main_spec``   — ``/root/reference/main.py:13-51`` verbatim (the scene that produced the
  committed ``render.png``). Python ints are kept as ints, exactly as main.py writes them.
* ``readme_spec`` — the README scene (``/root/reference/README.md:50-84``) translated to today's
  API: every shader ``NumpyShader(0.8, 1.0, 0.5, 0.05, 1.0, tex)``; ground ``TextureChecker``.
  This is BASELINE.json configs[0] / configs[1].
* ``random_spec`` — the seeded generator of SURVEY.md §8d (configs C3/C4/C5).
* ``orbit_position`` — C5's camera orbit.

Spec layout::

    {"spheres": [{"center": [x, y, z], "radius": r,
                  "shader": {"reflection_gain": .., "specular_gain": .., "specular_roughness": ..,
                             "iridescence_gain": .., "diffuse_gain": ..,
                             "texture": {"kind": "const" | "checker", "color": [r, g, b]}}}],
                  (or {"kind": "image", "texels": (H, W, 3) float colours} — ImageTexture)
     "lights": [{"kind": "point", "position": [x, y, z]},
                {"kind": "dome", "intensity": i, "color": [r, g, b]}],
     "camera": {"position": [x, y, z], "width": W, "height": H}}
"""

from __future__ import annotations

import copy
import math

import numpy as np


def _shader(reflection_gain, specular_gain, specular_roughness, iridescence_gain, diffuse_gain, texture):
    return {
        "reflection_gain": reflection_gain,
        "specular_gain": specular_gain,
        "specular_roughness": specular_roughness,
        "iridescence_gain": iridescence_gain,
        "diffuse_gain": diffuse_gain,
        "texture": texture,
    }


def _const(r, g, b):
    return {"kind": "const", "color": [r, g, b]}


def _checker():
    # TextureChecker's own colour is ignored by get_color (shader.py:29-32)
    return {"kind": "checker", "color": [1, 1, 1]}


def main_spec(width: int = 960, height: int = 540) -> dict:
    """``/root/reference/main.py:13-51``; default size is main.py's ``int(1920/2) x int(1080/2)``."""
    return {
        "spheres": [
            {"center": [0.55, 0.5, 3], "radius": 1.0,
             "shader": _shader(0.0, 0, 0.01, 0, 0.0, _const(1, 1, 1))},
            {"center": [-0.45, 0.1, 1], "radius": 0.4,
             "shader": _shader(0, 1, 0.1, 0.0, 0.0, _const(1, 0, 0))},
            {"center": [0, -99999.5, 0], "radius": 99999,
             "shader": _shader(0.0, 0.1, 0.5, 0.0, 1.0, _checker())},
        ],
        "lights": [
            {"kind": "point", "position": [-2, 1, 2]},
            {"kind": "dome", "intensity": 0.1, "color": [1, 1, 1]},
        ],
        "camera": {"position": [0, 0.2, -2], "width": int(width), "height": int(height)},
    }


def readme_spec(width: int = 1920, height: int = 1080) -> dict:
    """README scene, translated."""
    gains = (0.8, 1.0, 0.5, 0.05, 1.0)
    return {
        "spheres": [
            {"center": [0.55, 0.5, 3], "radius": 1.0, "shader": _shader(*gains, _const(1, 0, 1))},
            {"center": [-0.45, 0.1, 1], "radius": 0.4, "shader": _shader(*gains, _const(0.5, 0.5, 0.5))},
            {"center": [0, -99999.5, 0], "radius": 99999, "shader": _shader(*gains, _checker())},
        ],
        "lights": [
            {"kind": "point", "position": [5, 10, -10]},
            {"kind": "dome", "intensity": 0.1, "color": [1, 1, 1]},
        ],
        "camera": {"position": [0, 0.2, -2], "width": int(width), "height": int(height)},
    }


def random_spec(n_spheres: int, seed: int = 0, width: int = 3840, height: int = 2160) -> dict:
    """Seeded random scene of SURVEY.md §8d: PCG64 draws per sphere, in this order,
    r~U(0.1,0.5), cx~U(-4,4), cz~U(0.5,14), colour~U(0,1)^3, then the shader gains
    reflection~U(0,1), specular~U(0,1), roughness~U(0.05,0.9), iridescence~U(0,0.1),
    diffuse~U(0.3,1). Centre (cx, r-0.5, cz) rests the sphere on the ground. A checker ground
    sphere is appended; lights [PointLight(-2,4,-1), DomeLight(0.1, white)]; camera (0,0.2,-2)."""
    rng = np.random.default_rng(seed)
    spheres = []
    for _ in range(int(n_spheres)):
        r = float(rng.uniform(0.1, 0.5))
        cx = float(rng.uniform(-4, 4))
        cz = float(rng.uniform(0.5, 14))
        col = [float(v) for v in rng.uniform(0, 1, 3)]
        refl = float(rng.uniform(0, 1))
        spec = float(rng.uniform(0, 1))
        rough = float(rng.uniform(0.05, 0.9))
        irid = float(rng.uniform(0, 0.1))
        diff = float(rng.uniform(0.3, 1))
        spheres.append({"center": [cx, r - 0.5, cz], "radius": r,
                        "shader": _shader(refl, spec, rough, irid, diff, _const(*col))})
    spheres.append({"center": [0, -99999.5, 0], "radius": 99999,
                    "shader": _shader(0.0, 0.1, 0.5, 0.0, 1.0, _checker())})
    return {
        "spheres": spheres,
        "lights": [
            {"kind": "point", "position": [-2, 4, -1]},
            {"kind": "dome", "intensity": 0.1, "color": [1, 1, 1]},
        ],
        "camera": {"position": [0, 0.2, -2], "width": int(width), "height": int(height)},
    }


def orbit_position(frame: int, n_frames: int = 256) -> list:
    """C5 camera orbit: frame k at (sin θ, 0.2, -2 - cos θ), θ = 2πk/n (z stays < 0 because the
    reference screen is fixed at z=0, ``base.py:131-141``)."""
    theta = 2.0 * math.pi * frame / n_frames
    return [math.sin(theta), 0.2, -2.0 - math.cos(theta)]


def path_position(spec: dict, frame: int, n_frames: int = 256) -> list:
    """Frame k of the camera path through a config's own camera (the ``bench.py --gpus N``
    headline: rank r renders frame r, so frame 0 — rank 0, and the N = 1 line — is the config's
    frame itself). A circle of radius 1 in the horizontal plane, frame 0 at the camera and the
    centre one unit behind it: (cx + sin θ, cy, cz - 1 + cos θ), θ = 2πk/n. z stays ≤ cz, so a
    config camera in front of the reference's fixed screen (z < 0, ``base.py:131-141``) stays there."""
    cx, cy, cz = (float(v) for v in spec["camera"]["position"])
    theta = 2.0 * math.pi * frame / n_frames
    return [cx + math.sin(theta), cy, (cz - 1.0) + math.cos(theta)]


def rank_frame_spec(spec: dict, rank: int, n_frames: int = 256) -> dict:
    """The frame a rank of the weak-scaling headline renders: the config's own spec at rank 0
    (unchanged, so the N = 1 line is the single-GPU line), frame ``rank`` of ``path_position``
    elsewhere — every rank a distinct frame of one camera path, as ``render_image_pipeline`` renders
    one frame per call (``application.py:43-52``)."""
    if rank % n_frames == 0:
        return spec
    return with_camera(spec, path_position(spec, rank, n_frames))


def with_camera(spec: dict, position=None, width=None, height=None) -> dict:
    """Copy of ``spec`` with camera fields replaced."""
    out = copy.deepcopy(spec)
    if position is not None:
        out["camera"]["position"] = list(position)
    if width is not None:
        out["camera"]["width"] = int(width)
    if height is not None:
        out["camera"]["height"] = int(height)
    return out


CONFIGS = {
    # BASELINE.json configs, by index
    "C1": lambda: (readme_spec(960, 540), 3),
    "C2": lambda: (readme_spec(1920, 1080), 3),
    "C2main": lambda: (main_spec(1920, 1080), 3),
    "C3": lambda: (random_spec(16, 0, 3840, 2160), 4),
    "C4": lambda: (random_spec(64, 0, 7680, 4320), 5),
    "C5": lambda: (random_spec(16, 0, 1920, 1080), 3),
}


def build_scene(spec: dict):
    """Instantiate ``spec`` with this package's HIP-backend classes."""
    from python_ray_tracer_amd.domain import Camera, DomeLight, PointLight, Scene3D
    from python_ray_tracer_amd.infrastructure.hip import (
        HipRGBColor,
        HipShader,
        HipSphere,
        HipVector3D,
        ImageTexture,
        Texture,
        TextureChecker,
    )

    shapes = []
    for s in spec["spheres"]:
        sh = s["shader"]
        tex = sh["texture"]
        if tex["kind"] == "checker":
            texture = TextureChecker()
        elif tex["kind"] == "image":
            texture = ImageTexture(np.asarray(tex["texels"], dtype=np.float64))
        else:
            texture = Texture(HipRGBColor(*tex["color"]))
        shader = HipShader(sh["reflection_gain"], sh["specular_gain"], sh["specular_roughness"],
                           sh["iridescence_gain"], sh["diffuse_gain"], texture)
        shapes.append(HipSphere(HipVector3D(*s["center"]), s["radius"], shader))
    lights = []
    for li in spec["lights"]:
        if li["kind"] == "point":
            lights.append(PointLight(HipVector3D(*li["position"])))
        else:
            lights.append(DomeLight(li["intensity"], HipRGBColor(*li["color"])))
    cam = spec["camera"]
    return Scene3D(shapes, lights, Camera(HipVector3D(*cam["position"]), cam["width"], cam["height"]))
