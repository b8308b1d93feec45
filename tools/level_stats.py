"""Per-level ray / hit / wave-occupancy counters of the fast kernel for the bench configurations.

    python tools/level_stats.py [C2 C2main C3 C4 C5]

lane utilisation at a level = rays (or hits) / (64 x waves that executed the stage).
"""

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import HipRenderer  # noqa: E402


def main():
    for cfg in sys.argv[1:] or ["C2", "C2main", "C3", "C4"]:
        spec, B = scenes.CONFIGS[cfg]()
        r = HipRenderer(max_bounces=B, color_dtype=torch.float32, collect_stats=True)
        r.render_tile(scenes.build_scene(spec))
        s = r.stats()
        print(f"== {cfg}: B={B} S={len(spec['spheres'])} pixels={s['pixels']} deferred={s['deferred']}")
        tot_wt = tot_ws = tot_r = tot_h = 0
        for k, (rays, hits, wt, ws) in enumerate(zip(s["rays"], s["hits"], s["waves_traced"], s["waves_shaded"])):
            print(f"  level {k}: rays {rays:>10,} waves {wt:>8,} ({rays / max(64 * wt, 1):5.1%})   "
                  f"hits {hits:>10,} waves {ws:>8,} ({hits / max(64 * ws, 1):5.1%})")
            tot_wt += wt
            tot_ws += ws
            tot_r += rays
            tot_h += hits
        print(f"  all    : trace lane-util {tot_r / max(64 * tot_wt, 1):5.1%}   shade lane-util {tot_h / max(64 * tot_ws, 1):5.1%}")


if __name__ == "__main__":
    main()
