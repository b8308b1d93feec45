"""Time per step of the row-tiled pipeline (distributed.TileGather), one GPU.

    python tools/tiles_ab.py --config C2 --heights 1080,136,8

On a one-rank RCCL group, frames of the config's scene at each height (136 rows of 1920 is one
rank's part of the 1080p frame at N = 8; 8 rows leave almost no GPU work, so their step time is the
host's cost of a step) go through the two-slot pipeline of bench.py's tiles mode (submit k, finish
k-1). Prints µs per step (best and median of R rounds) and checks the frames against single
renders. (Session r3k also timed a TileGather with per-slot streams and a side stream for the
assembly: its host cost per step was 87 µs against 49 µs, so it was removed.)
"""

from __future__ import annotations

import argparse
import json
import socket
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--heights", default="1080,136")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default=None)
    ap.add_argument("--profile", action="store_true", help="cProfile the steps of the last height")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.distributed import TileGather
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dev = torch.device("cuda", 0)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    spec, B = scenes.CONFIGS[a.config]()
    res = {}
    for H in [int(v) for v in a.heights.split(",")]:
        sp = json.loads(json.dumps(spec))
        sp["camera"]["height"] = H
        scene = scenes.build_scene(sp)
        W = sp["camera"]["width"]
        r = HipRenderer(max_bounces=B, color_dtype=torch.float32, device=dev)
        want = r.render_tile(scene, out="u8").clone()
        variants = {}
        for name in ("pipeline",):
            tg = TileGather(r, W, H, row_block=8, out="u8", slots=2)
            state = {"k": 0, "open": None, "last": None}

            def step(tg=tg, state=state):
                slot = state["k"] % 2
                tg.submit(scene, slot)
                if state["open"] is not None:
                    state["last"] = tg.finish(state["open"])
                state["open"] = slot
                state["k"] += 1

            def drain(tg=tg, state=state):
                if state["open"] is not None:
                    state["last"] = tg.finish(state["open"])
                    state["open"] = None
            variants[name] = (step, drain, state)
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for name, (step, drain, state) in variants.items():
                for _ in range(5):
                    step()
                drain()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step()
                drain()
                torch.cuda.synchronize()
                times[name].append((time.perf_counter() - t0) / a.steps * 1e6)
                assert torch.equal(state["last"], want), (H, name)
        if a.profile and H == int(a.heights.split(",")[-1]):
            import cProfile
            import pstats

            step, drain, _ = variants["pipeline"]
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(a.steps):
                step()
            drain()
            pr.disable()
            torch.cuda.synchronize()
            pstats.Stats(pr).sort_stats("tottime").print_stats(25)
        for name, ts in times.items():
            ts.sort()
            res[f"{W}x{H} {name}"] = {"best_us_per_step": round(ts[0], 2), "median_us_per_step": round(ts[len(ts) // 2], 2)}
            print(f"{a.config} {W}x{H} {name:10s} best {ts[0]:8.2f} us/step  median {ts[len(ts) // 2]:8.2f}", flush=True)
    dist.destroy_process_group()
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
