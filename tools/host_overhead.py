"""Host (Python) cost of one bench step, measured on the GPU box.

    python tools/host_overhead.py --config C2 [--profile]

Times N back-to-back calls of the bench's step (raytrace_scene through the public API) without
synchronising: while the GPU is slower than the host, the wall time per call is the host's cost
(the launches queue up); a host cost near the kernel time means the GPU starves between steps.
"""

import argparse
import cProfile
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import HipRenderer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    scene = scenes.build_scene(spec)
    r = HipRenderer(max_bounces=B, color_dtype=torch.float32)

    def step():
        return r.raytrace_scene(scene.camera.position, r.get_ray_directions(scene.camera), scene)

    def tile():
        return r.render_tile(scene)

    for fn, name in ((step, "raytrace_scene(get_ray_directions)"), (tile, "render_tile")):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:40s} host {1e6 * (t1 - t0) / a.calls:8.1f} us/call   wall {1e6 * (t2 - t0) / a.calls:8.1f} us/call")
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.calls):
            step()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
