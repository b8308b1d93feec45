"""A/B: eager frames against HIP-graph replays of the same frames, one process.

    python tools/graph_ab.py --config C2 [--frames-per-graph 1,8] [--tiles]

Per variant: K timed frames between synchronisations, end-to-end µs per frame (host launch cost,
the fast kernel, the tie kernel and the gaps between them), best of R rounds, variants
interleaved. "eager": HipRenderer.render_tile(scene, into=buf) per frame; "graph xF": F such calls
captured into one torch.cuda.CUDAGraph, replayed K/F times. With --tiles, the same for one
TileGather step (render into the gather buffer, gather over a one-rank nccl group, assemble_rows),
eager only.
Every replayed frame is checked against the eager frame (bit equality).
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
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--frames-per-graph", default="1,8")
    ap.add_argument("--tiles", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    spec, B = scenes.CONFIGS[a.config]()
    scene = scenes.build_scene(spec)
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    dev = torch.device("cuda", 0)
    r = HipRenderer(max_bounces=B, color_dtype=torch.float32, device=dev)
    buf = torch.empty((3, W * H), dtype=torch.float32, device=dev)
    want = r.render_tile(scene).clone()

    variants = {}

    def eager():
        r.render_tile(scene, into=buf)
    variants["eager"] = (eager, 1)

    def eager_new_out():
        return r.render_tile(scene)
    variants["eager new out"] = (eager_new_out, 1)

    def bench_step():  # bench.py's step: the public API, a new output every frame
        return r.raytrace_scene(scene.camera.position, r.get_ray_directions(scene.camera), scene)
    variants["bench step"] = (bench_step, 1)

    s = torch.cuda.Stream(device=dev)
    keep = []
    for F in [int(v) for v in a.frames_per_graph.split(",")]:
        bufs = [torch.empty_like(buf) for _ in range(F)]
        r.render_tile(scene, into=bufs[0])  # workspace sized, scene uploaded: nothing allocates in capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for f in range(F):
                    r.render_tile(scene, into=bufs[f])
        g.replay()
        torch.cuda.synchronize()
        ok = all(torch.equal(b, want) for b in bufs)
        # the graph writes into bufs on every replay: keep them (and the graph) alive. (Rebinding
        # bufs for the next F freed the previous graph's outputs, which the next capture's
        # empty_cache() returned to the driver: its replays then wrote to unmapped memory — the
        # illegal-address faults of sessions r3g and r3g2.)
        keep.append((g, bufs))
        variants[f"graph x{F}"] = (g.replay, F)
        print(f"graph x{F}: captured, frames equal eager: {ok}", flush=True)

    if a.tiles:
        import torch.distributed as dist

        from python_ray_tracer_amd.distributed import TileGather

        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        tg = TileGather(r, W, H, row_block=8, out="u8", slots=1)
        want_u8 = r.render_tile(scene, out="u8").clone()

        def tiles_eager():
            return tg.render(scene)
        variants["tiles eager"] = (tiles_eager, 1)
        got = tiles_eager()
        torch.cuda.synchronize()
        print("tiles eager frame equal:", torch.equal(got, want_u8), flush=True)
        # A graph-captured gather replayed between eager gathers on the same communicator faulted
        # the GPU (illegal address, session r3g): the tiles step is measured eager only.

    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for name, (fn, F) in variants.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            n = max(1, a.frames // F)
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / (n * F) * 1e6)
    out = {}
    for name, ts in res.items():
        ts.sort()
        out[name] = {"best_us_per_frame": round(ts[0], 2), "median_us_per_frame": round(ts[len(ts) // 2], 2)}
        print(f"{a.config} {name:12s} best {ts[0]:8.2f} us/frame  median {ts[len(ts) // 2]:8.2f}", flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps({"config": a.config, "variants": out}, indent=1))


if __name__ == "__main__":
    main()
