"""Render a config's scene with no bounce cap (the reference default) repeatedly, for a rocprofv3
kernel trace of the three launches (first pass, continuation pass, general kernel).

    rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/unbounded_probe.py --config C2main
"""

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import HipRenderer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2main")
    ap.add_argument("--frames", type=int, default=30)
    a = ap.parse_args()
    spec, _ = scenes.CONFIGS[a.config]()
    scene = scenes.build_scene(spec)
    r = HipRenderer(color_dtype=torch.float32)  # max_bounces=None
    for _ in range(a.frames):
        r.render(scene)
    torch.cuda.synchronize()
    print("ok", a.config, a.frames)


if __name__ == "__main__":
    main()
