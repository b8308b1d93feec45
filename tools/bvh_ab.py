"""A/B of culling-tree builds (scene_pack.BVH_LEAF / BVH_NODE_COST) on the GPU, one process.

    python tools/bvh_ab.py --configs C3,C4,C5 --variants 8:-,16:-,32:-,64:2,64:4 --out gpurun_out/bvh.json

A variant "leaf:cost" sets BVH_LEAF = leaf and BVH_NODE_COST = cost ("-" = None: always split above
the leaf size). For every config and variant: the kernel's executed-work counters (sphere and node
tests, STATS launch), the fast kernel's mean time over K launches (the library's HIP events, the
variants interleaved round-robin so clock drift spreads evenly) and a bit-equality check of the frame
against the first variant's (culling must not change a bit).
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3,C4,C5")
    ap.add_argument("--variants", default="8:-,16:-,32:-,64:2,64:4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--per-round", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer
    from python_ray_tracer_amd.infrastructure.hip import _lib as L
    from python_ray_tracer_amd.infrastructure.hip import scene_pack as P

    variants = []
    for v in a.variants.split(","):
        leaf, cost = v.split(":")
        variants.append((int(leaf), None if cost == "-" else float(cost)))
    res = {}
    for cfg in a.configs.split(","):
        spec, B = scenes.CONFIGS[cfg]()
        F = 8 if cfg == "C5" else 1  # C5: a batch of orbit frames per launch, like the bench
        frames = ([scenes.build_scene(scenes.with_camera(spec, scenes.orbit_position(f, 256))) for f in range(F)]
                  if F > 1 else [scenes.build_scene(spec)])
        rows = []
        ref = None
        runs = []
        for leaf, cost in variants:
            P.BVH_LEAF, P.BVH_NODE_COST = leaf, cost
            P._pack_static.cache_clear()
            r = HipRenderer(max_bounces=B, color_dtype=torch.float32)
            rs = HipRenderer(max_bounces=B, color_dtype=torch.float32, collect_stats=True)
            step = (lambda r=r: r.render_batch(frames)) if F > 1 else (lambda r=r: r.render_tile(frames[0]))
            img = step()
            (rs.render_batch(frames) if F > 1 else rs.render_tile(frames[0]))
            st = rs.stats()
            nodes = int((rs.scene_blob(frames[0])[0][L.H_NNODES]).item())
            same = True if ref is None else bool(torch.equal(img, ref))
            if ref is None:
                ref = img
            row = {"leaf": leaf, "node_cost": cost, "tree_nodes": nodes, "sphere_tests": st["sphere_tests"],
                   "node_tests": st["node_tests"], "identical": same, "kernel_us": []}
            rows.append(row)
            runs.append((row, step))
        for _ in range(a.rounds):
            for row, step in runs:
                step()
                torch.cuda.synchronize()
                L.profile_sample(1)
                L.profile_enable(a.per_round)
                for _ in range(a.per_round):
                    step()
                ms, n = L.profile_collect()
                L.profile_enable(0)
                row["kernel_us"].append(ms / max(n, 1) * 1e3)
        for row in rows:
            ks = sorted(row["kernel_us"])
            row["kernel_us_median"] = round(ks[len(ks) // 2], 2)
            row["kernel_us"] = [round(k, 2) for k in row["kernel_us"]]
        base = rows[0]["kernel_us_median"]
        for row in rows:
            row["vs_first"] = round(row["kernel_us_median"] / base - 1, 4)
            print(cfg, json.dumps({k: row[k] for k in ("leaf", "node_cost", "tree_nodes", "sphere_tests", "node_tests",
                                                        "identical", "kernel_us_median", "vs_first")}), flush=True)
        res[cfg] = rows
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
