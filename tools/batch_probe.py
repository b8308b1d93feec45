"""Per-frame kernel time of a config rendered 1, 4, 16 times per launch (rtx_render_frames).

    python tools/batch_probe.py --config C2

Many copies of one frame in one launch amortise the grid's ramp-up and drain, so the per-frame
time at 16 copies approximates a tail-free single frame: the gap to the 1-copy time is what the
single-frame launch loses to its tail.
"""

import argparse
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import HipRenderer  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--copies", default="1,4,16")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    scene = scenes.build_scene(spec)
    r = HipRenderer(max_bounces=B, color_dtype=torch.float32)
    for c in (int(x) for x in a.copies.split(",")):
        batch = [scene] * c
        for _ in range(3):
            r.render_batch(batch)
        torch.cuda.synchronize()
        per = []
        for _ in range(5):
            L.profile_enable(a.iters)
            for _ in range(a.iters):
                r.render_batch(batch)
            ms, n = L.profile_collect()
            L.profile_enable(0)
            per.append(ms / max(n, 1) / c * 1e3)
        print(f"{a.config} copies {c:3d}: kernel {statistics.median(per):8.2f} us/frame")


if __name__ == "__main__":
    main()
