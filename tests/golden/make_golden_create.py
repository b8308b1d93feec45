"""Known answers for ``NumpyShader.create`` (shader.py:63-112) called directly, the Shader plugin
surface (application.py:35-40), by running the REFERENCE in the build container:

    python tests/golden/make_golden_create.py      -> create_kat.npz, create_kat.json

For a few scenes, the camera rays of a small frame are intersected with one shape (its own
``NumpySphere.intersect``, shape.py:28-51); the rays it hits — nearest or not: create shades what
it is handed — go to ``shape.shader.create(shape, scene, O, D, t, renderer)``. The renderer is the
reference ``NumpyRenderer`` under the same bounce-capping wrapper as make_golden.py, entered at
depth 1 so that the reflected rays are level 1 (levels 0..B shaded). Stored: the rays, t, and
the float64 colour.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent.parent))

import make_golden as G  # noqa: E402  (the reference import shim, ref_scene, CappedRenderer)

from python_ray_tracer_amd import scenes as S  # noqa: E402


def main():
    R = G.R
    V = R["NumpyVector3D"]
    cases = {
        "readme_s0_B3": (S.readme_spec(48, 27), 0, 3),
        "readme_ground_Binf": (S.readme_spec(48, 27), 2, None),
        "main_s1_B2": (S.main_spec(40, 24), 1, 2),
        "rand16_s9_B4": (S.random_spec(16, 0, 96, 54), 9, 4),
        "rand16_s12_Binf": (S.random_spec(16, 0, 96, 54), 12, None),
        # create called on ANOTHER shape's shader: the hit is shaded with that shader's parameters,
        # the reflections are traced through the unchanged scene (shader.py:73-112, :152)
        "rand16_s9_shader3_B3": (S.random_spec(16, 0, 96, 54), 9, 3, 3),
        "readme_ground_shader0_Binf": (S.readme_spec(48, 27), 2, None, 0),
        "rand16_s12_shader16_B2": (S.random_spec(16, 0, 96, 54), 12, 2, 16),
    }
    arrays, meta = {}, {"note": "reference NumpyShader.create on the rays that hit the shape", "cases": {}}
    for name, (spec, si, B, *other) in cases.items():
        scene = G.ref_scene(spec)
        rend = G.CappedRenderer(B)
        dirs = rend.get_ray_directions(scene.camera)
        shape = scene.shapes[si]
        t = np.asarray(shape.intersect(scene.camera.position, dirs))
        hit = t != 1.0e39
        D = V(dirs.x[hit], dirs.y[hit], dirs.z[hit])
        O = scene.camera.position
        rend.depth = 1  # inside level 0's raytrace_scene: the reflection is level 1
        shader = scene.shapes[other[0]].shader if other else shape.shader
        col = shader.create(shape, scene, O, D, t[hit], rend)
        n = int(hit.sum())
        out = np.stack([np.broadcast_to(np.asarray(c, dtype=np.float64), (n,)) for c in col.components()])
        arrays[f"{name}_dirs"] = np.stack([D.x, D.y, D.z])
        arrays[f"{name}_t"] = t[hit]
        arrays[f"{name}_rgb"] = out
        meta["cases"][name] = {"spec": spec, "shape": si, "max_bounces": B, "n": n,
                               "origin": [float(O.x), float(O.y), float(O.z)],
                               "shader_of": other[0] if other else si}
        print(name, n, "rays")
    np.savez_compressed(HERE / "create_kat.npz", **arrays)
    (HERE / "create_kat.json").write_text(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
