"""Image-textured scene: the fast kernel's texturing build (RTX_F_IMAGES, HipRenderer(fast_textures=True))
against deferring the textured pixels to the general kernel (fast_textures=False).

    python tools/texture_ab.py [--width 1920 --height 1080 --bounces 3 --iters 50] [--json-out F]

Scene: the README scene plus two image-textured spheres (a mirror-ish one and a diffuse one, as
tests/test_gpu_parity.py's _textured_spec). Frames of the two renderers must be bit-identical; the
time per frame is wall clock over synchronised batches of renders (fast kernel + general kernel),
alternated, median of rounds.
"""

from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import HipRenderer  # noqa: E402


def textured_spec(W, H):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(40, 64, 3)).astype(np.float64) / 255.0
    spec = scenes.readme_spec(W, H)
    spec["spheres"].insert(0, {"center": [-0.9, 0.2, 2.0], "radius": 0.6,
                               "shader": {"reflection_gain": 0.0, "specular_gain": 0.0, "specular_roughness": 0.5,
                                          "iridescence_gain": 0.0, "diffuse_gain": 1.0,
                                          "texture": {"kind": "image", "texels": img}}})
    spec["spheres"].insert(1, {"center": [1.2, 0.0, 1.5], "radius": 0.5,
                               "shader": {"reflection_gain": 0.5, "specular_gain": 0.7, "specular_roughness": 0.2,
                                          "iridescence_gain": 0.05, "diffuse_gain": 0.8,
                                          "texture": {"kind": "image", "texels": img[::-1].copy()}}})
    return spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--json-out")
    a = ap.parse_args()
    scene = scenes.build_scene(textured_spec(a.width, a.height))
    rs = {"fast_textures": HipRenderer(max_bounces=a.bounces, color_dtype=torch.float32),
          "deferred": HipRenderer(max_bounces=a.bounces, color_dtype=torch.float32, fast_textures=False)}
    bufs = {k: torch.empty((3, a.width * a.height), dtype=torch.float32, device="cuda") for k in rs}
    for k, r in rs.items():
        for _ in range(3):
            r.render_tile(scene, into=bufs[k])
    torch.cuda.synchronize()
    if not torch.equal(bufs["fast_textures"], bufs["deferred"]):
        raise AssertionError("texturing build and deferral differ")
    times = {k: [] for k in rs}
    for _ in range(a.rounds):
        for k, r in rs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                r.render_tile(scene, into=bufs[k])
            torch.cuda.synchronize()
            times[k].append((time.perf_counter() - t0) / a.iters * 1e6)
    res = {"scene": f"README scene + 2 image-textured spheres, {a.width}x{a.height}, {a.bounces} bounces, f32",
           "us_per_frame_median": {k: round(statistics.median(v), 2) for k, v in times.items()},
           "rounds": {k: [round(x, 2) for x in v] for k, v in times.items()}, "frames_identical": True}
    print(json.dumps(res))
    if a.json_out:
        Path(a.json_out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
