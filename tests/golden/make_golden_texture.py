"""Known answers for the image-texture mapping of the reference's ``NumpyTexturedSphere``
(shape.py:57-90), by running the REFERENCE in the build container:

    python tests/golden/make_golden_texture.py     -> texture_kat.json

The reference class cannot render (its shader is an RGB colour, shape.py:64), but its
``diffusecolor`` runs: called with ONE point it returns that point's texel (with several points it
averages them into one colour, shape.py:81-90). A small uint8 image is written to a temporary PNG,
loaded by the reference constructor (shape.py:64-65), and ``diffusecolor`` is evaluated at points on
the sphere — random directions plus the poles, the u seam (z = 0, x < 0) and the texel edges'
neighbourhood. Stored: the image, the sphere, the points and the reference's texel colours.
"""

from __future__ import annotations

import json
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent.parent))

import make_golden as G  # noqa: E402  (the reference import shim)


def main():
    from PIL import Image

    sys.path.insert(0, str(G.REF))
    from ray_tracer.infrastructure.numpy.shape import NumpyTexturedSphere

    V = G.R["NumpyVector3D"]
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, size=(9, 13, 3), dtype=np.uint8)
    center, radius = [0.3, -0.2, 2.5], 0.8
    dirs = [rng.normal(size=3) for _ in range(300)]
    dirs += [np.array(v, dtype=float) for v in ([0, 1, 0], [0, -1, 0], [-1, 0, 0], [1, 0, 0], [0, 0, 1], [0, 0, -1],
                                                [-1, 0, 1e-17], [-1, 0, -1e-17], [0.3, 0.9, -0.2])]
    kat = {"image": img.tolist(), "center": center, "radius": radius, "points": [], "rgb": []}
    with tempfile.TemporaryDirectory() as d:
        path = Path(d) / "tex.png"
        Image.fromarray(img).save(path)
        sph = NumpyTexturedSphere(V(*center), radius, path)
        for n in dirs:
            n = n / np.linalg.norm(n)
            p = [center[k] + radius * float(n[k]) for k in range(3)]
            c = sph.diffusecolor(V(*p))
            kat["points"].append(p)
            kat["rgb"].append([float(c.x), float(c.y), float(c.z)])
    (HERE / "texture_kat.json").write_text(json.dumps(kat))
    print(len(kat["points"]), "points")


if __name__ == "__main__":
    main()
