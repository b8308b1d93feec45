"""Benchmark: Mpixels/s of the render path (BASELINE.json metric) on 1..N MI355X.

    python bench.py --gpus N --steps K --warmup W [--config C2] [--mode frames|tiles]

A *step* is one frame of the configuration through the public API — ``HipRenderer.raytrace_scene(
camera.position, get_ray_directions(camera), scene)``: scene packing (cached by content), primary
ray generation, nearest hit, shadow rays, shading and every reflection level up to the cap, with the
unclipped colour left in HBM (float32 [3, W*H]). PNG encoding is not part of a step.

Default workload: BASELINE.json configs[1] — the README scene at 1920x1080, 3 reflection bounces.
``--mode frames`` (the default at every N, weak scaling): every rank renders whole frames, no
collective in the loop (the frame sharding of config C5), so N=1 and N>1 lines measure
the same code path and output format. Rank r renders frame r of a camera path through the config's
camera (``scenes.rank_frame_spec``): rank 0 the config's own frame, so the N = 1 line is unchanged,
and N ranks render N distinct frames per step. The top-level ``strong_scaling`` object is the
row-tiled C4 frame (below) with its measured speed-up over one GPU and its gather per link. ``--mode tiles`` (strong scaling): every rank renders its
interleaved row tile of ONE frame and the uint8 tiles are gathered to rank 0 (RCCL) every step; the
default line carries it at every N as ``secondary.tiles_u8`` (the config) and ``secondary.c4_tiles``
(C4, 7680x4320), on a one-rank process group at N=1.

Timing: W untimed warm-up steps, then K steps bracketed by barrier + synchronize, max over ranks.
The dominant kernel's own time is measured live with HIP events recorded by the library on the
launch stream (rtx_profile_*) around one launch in --prof-every of the timed region, for the
roofline (timing a launch costs stream time, so timing every launch would depress `value`). Rank 0 also times the CPU oracle (NumPy float64,
single core) on a bounded sample of the same workload.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

# MI355X peaks (MI355X_MICROARCH.md; FP64 vector = half the FP32 vector rate, datasheet 78.6 TF)
PEAK_FP64_TFLOPS = 78.6
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--ramp-ms", type=float, default=200.0,
                    help="untimed steps for this long before the warm-up steps: the GPU leaves its idle clock "
                         "state (C2: 63.6 us kernel after 20 warm-up steps, 59.0 us from ~500 on, "
                         "profiles/r3_ramp.json); the timed region is still exactly --steps steps")
    ap.add_argument("--config", default="C2", help="C1|C2|C2main|C3|C4|C5 (python_ray_tracer_amd/scenes.py)")
    ap.add_argument("--mode", default="frames", choices=["frames", "tiles"],
                    help="frames (default: every rank renders whole frames, weak scaling) or tiles (row tiles + "
                         "RCCL gather of one frame, strong scaling)")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--out", default=None, choices=["f32", "f64", "u8"],
                    help="frame format left in HBM (default f32; u8 in tiles mode: the gathered frame is the "
                         "uint8 image save_image writes)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the tiles-mode (row tiles + gather) measurements of the config and of C4")
    ap.add_argument("--cpu-procs", type=int, default=14,
                    help="processes of the row-tiled all-cores CPU baseline (the box's CPU share is 16 cores, and "
                         "at most 16 processes may hold the GPU open: importing torch opens it in every worker, "
                         "so 14 workers + this process)")
    ap.add_argument("--frames-per-step", type=int, default=1,
                    help="frames mode: render this many orbit frames of the config (C5 camera path, "
                         "SURVEY.md 8d) per step in ONE launch (rtx_render_frames)")
    ap.add_argument("--bounces", type=int, default=None,
                    help="override the config's bounce cap (-1: unbounded, HipRenderer()'s default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline time budget (0: skip)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--prof-every", type=int, default=10,
                    help="time the dominant kernel with HIP events on one launch in this many (timing a launch "
                         "costs stream time; 1 = every launch)")
    ap.add_argument("--emulate-parts", default=None, metavar="N,N,...",
                    help="one GPU: time every part p of render_tile(scene, row_block, N, p) for each N (the compute "
                         "side of the N-GPU row-tiled frame) and assemble_rows of N parts; prints one JSON line "
                         "(metric: per-part kernel time) instead of the bench line")
    ap.add_argument("--no-tile-order", action="store_true",
                    help="camera launches keep the bottom-up tile order instead of the longest-first order "
                         "HipRenderer learns from its first launch of a scene (A/B)")
    ap.add_argument("--loopback", action="store_true",
                    help="tiles mode on one GPU: a one-rank RCCL group whose plan still sends its tile through "
                         "RCCL (to itself) and assembles it, two frames in flight: how the gather's RCCL kernels "
                         "share the GPU with the next frame's render")
    ap.add_argument("--comm-reserve", type=int, default=None,
                    help="tiles mode: block slots a gathering plan's persistent renders leave free for the RCCL "
                         "kernels of the previous frame (default distributed.COMM_RESERVE_BLOCKS)")
    ap.add_argument("--rows", action="store_true",
                    help="tiles mode: move each row block straight into the root's frame (RTX_TILES_ROWS) instead "
                         "of gathering whole tiles and assembling them on the root (A/B)")
    ap.add_argument("--shares", default=None, metavar="ROOT_RUN,RUN",
                    help="--emulate-parts: the root renders ROOT_RUN parts and every other rank RUN parts of the "
                         "interleave (default distributed.ROOT_SHARES by N)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one rank per GPU); gloo is a test mode for ranks sharing a GPU")
    return ap.parse_args()


def main():
    args = parse()
    if args.out is None:
        args.out = "u8" if args.mode == "tiles" else "f32"
    import numpy as np
    import torch
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer
    from python_ray_tracer_amd.infrastructure.hip import _lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one process per GPU; --backend gloo (test mode) lets several ranks share fewer GPUs
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} visible GPUs")
    local_dev = local % max(ndev, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")

    spec, B = scenes.CONFIGS[args.config]()
    if args.bounces is not None:
        B = None if args.bounces < 0 else args.bounces
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    scene = scenes.build_scene(spec)
    dtype = torch.float64 if args.out == "f64" else torch.float32
    r = HipRenderer(max_bounces=B, color_dtype=dtype, device=dev, learn_tile_order=not args.no_tile_order)

    if args.emulate_parts:
        line = emulate_parts(args, r, scene, spec, B, [int(v) for v in args.emulate_parts.split(",")])
        print(json.dumps(line))
        if args.json_out:
            Path(args.json_out).write_text(json.dumps(line) + "\n")
        return

    F = max(1, args.frames_per_step)
    own = scene  # the frame this rank renders (frames mode, F = 1)
    if args.mode == "frames" and F > 1:
        # rank r renders orbit frames r*F .. r*F+F-1 of a 256-frame orbit (C5 camera path)
        batch = [scenes.build_scene(scenes.with_camera(spec, scenes.orbit_position(rank * F + f, 256)))
                 for f in range(F)]

        def step():
            return r.render_batch(batch, out="u8" if args.out == "u8" else None)
        px_per_step = W * H * F * world
    elif args.mode == "frames":
        # rank r renders frame r of the camera path through the config's camera (scenes.rank_frame_spec):
        # rank 0 the config's frame itself (the N = 1 line), every other rank a distinct frame, so the
        # N-GPU line renders N different frames per step and moves nothing between GPUs
        own = scene if rank == 0 else scenes.build_scene(frame_spec_for_rank(spec, rank))

        def step():
            if args.out == "u8":
                return r.render_tile(own, out="u8")
            return r.raytrace_scene(own.camera.position, r.get_ray_directions(own.camera), own)
        px_per_step = W * H * world
    else:
        # strong scaling: every rank renders its interleaved row tile of ONE frame into a gather
        # buffer, one gather to rank 0, one device un-permute there; two slots, so the gather of
        # frame k overlaps the render of frame k+1 (python_ray_tracer_amd/distributed.py)
        if args.loopback and world == 1 and not dist.is_initialized():
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                    device_id=dev)
        step, drain = tiles_stepper(r, scene, world, args.row_block, "u8" if args.out == "u8" else None,
                                    loopback=args.loopback, comm_reserve=args.comm_reserve,
                                    rows=args.rows)
        px_per_step = W * H

    def barrier():  # every rank's queued GPU work done, then all ranks meet
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    if args.mode != "tiles":
        def drain():
            return None

    # clock ramp (untimed): steps until --ramp-ms has passed, synchronising every 32 so the host does
    # not queue far ahead; then the W warm-up steps and the timed region as the contract says
    step()  # the first call loads the code object and uploads the scene: not part of the ramp's time
    drain()
    torch.cuda.synchronize(dev)
    n_ramp = 1
    t_ramp = time.perf_counter()
    while (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
        step()
        n_ramp += 1
        if n_ramp % 32 == 0:
            drain()
            torch.cuda.synchronize(dev)
    drain()
    barrier()
    for _ in range(args.warmup):
        step()
    drain()
    barrier()
    # the library times launches every-1, 2*every-1, ...: at least one of the timed region
    every = max(1, min(args.prof_every, args.steps))
    L.profile_sample(every)
    L.profile_enable(args.steps)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, kern_n = L.profile_collect()
    L.profile_enable(0)
    L.profile_sample(1)
    if world > 1:  # the job takes as long as its slowest rank
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # algorithmic work of one launch, from the kernel's own counters (checked against the oracle in
    # tests/test_gpu_parity.py): 15 flops / primary ray, 20 / ray-sphere test, 200 / shaded hit
    rs = HipRenderer(max_bounces=B, color_dtype=dtype, device=dev, collect_stats=True)
    if args.mode == "frames" and F > 1:
        rs.render_batch(batch)
        n_px_launch = W * H * F
    elif args.mode == "frames" or world == 1:
        rs.render_tile(own)
        n_px_launch = W * H
    else:
        from python_ray_tracer_amd.tiling import n_local_rows

        rs.render_tile(scene, args.row_block, world, rank)
        n_px_launch = W * n_local_rows(H, args.row_block, world, rank)
    st = rs.stats()
    S = len(spec["spheres"])
    R_tr, R_sh = sum(st["rays"]), sum(st["hits"])
    flops = 15 * n_px_launch + 20 * S * (R_tr + R_sh) + 200 * R_sh
    # the same model over the work the fast kernel actually executed: its ray-sphere tests (the
    # culling tree skips most of the S per ray at C3/C4; the shadow loop stops at the first
    # occluder), its culling-node tests (~22 flops: 6 subtractions, 6 products, 10 min/max/compare)
    # and its reflected-ray beam tests (a lane's cone test of one sphere, round 6: 34 f64 operations
    # and 3 compares, rtx_kernels.hip wave_beam; until round 5 priced as two node tests)
    flops_exec = (15 * n_px_launch + 20 * st["sphere_tests"] + 22 * st["node_tests"] + 37 * st["beam_tests"]
                  + 200 * R_sh)
    out_bytes = {"f32": 12, "f64": 24, "u8": 3}[args.out]
    alg_bytes = out_bytes * n_px_launch + 8 * len(r.scene_blob(scene)[0]) * F  # framebuffer write + scene read
    kern_avg_s = kern_ms / 1e3 / max(kern_n, 1)
    achieved_tflops = flops / kern_avg_s / 1e12
    achieved_exec = flops_exec / kern_avg_s / 1e12
    achieved_gbs = alg_bytes / kern_avg_s / 1e9
    # A scene with a culling tree (C3, C4, C5) skips most of the tests the reference performs: the
    # headline fraction is then the executed-work one (the kernel's efficiency), and the §8d figure,
    # which prices every reference test, is kept as reference_equivalent.
    culled = st["node_tests"] > 0
    head_tflops, head_flops = (achieved_exec, flops_exec) if culled else (achieved_tflops, flops)

    traffic = None
    pmc = REPO / "profiles" / "pmc_traffic.json"
    # the PMC figures are whole-frame launches with float32 output on one GPU (tools/gpu_pmc.sh):
    # a row tile or another output format is a different launch, reported as unmeasured
    if pmc.exists() and world == 1 and args.out == "f32":
        try:
            d = json.loads(pmc.read_text())
            traffic = d.get(args.config, {}).get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    out_path = output_path_times(r, scene) if rank == 0 else None

    secondary = None
    if not args.no_secondary and args.frames_per_step == 1 and args.mode == "frames":
        secondary = secondary_tiles(args, r, scene, world, dev, coll_dev)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(spec, B, args.cpu_seconds)
        cpu = cpu_baseline_or_error(spec, B, args.cpu_procs, args.cpu_seconds, cpu)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = px_per_step * args.steps / elapsed / 1e6
        line = {
            "metric": "Mpixels/sec @1920x1080, 3 reflection bounces" if args.config in ("C2", "C2main") and B == 3
            else f"Mpixels/sec ({args.config}, {'unbounded' if B is None else B} bounces)",
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ramp": {"ms": args.ramp_ms, "steps": n_ramp,
                     "note": "untimed steps before the warm-up steps, bringing the GPU out of its idle clock "
                             "state (profiles/r3_ramp.json)"},
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "frames" else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "output_dtype": {"f32": "f32 SoA", "f64": "f64 SoA", "u8": "u8 HWC"}[args.out],
            "data": "synthetic",
            "config": {"workload": f"{args.config}: " + {
                "C1": "README scene 960x540",
                "C2": "README scene (BASELINE configs[1]) 1920x1080",
                "C2main": "main.py scene 1920x1080",
                "C3": "16 random spheres + checker ground 3840x2160 seed 0",
                "C4": "64 random spheres + checker ground 7680x4320 seed 0",
                "C5": "16 random spheres 1920x1080 seed 0"}[args.config]
                + (", unbounded bounces" if B is None else f", {B} bounces"),
                "width": W, "height": H, "max_bounces": B, "spheres": S, "output": args.out,
                "mode": args.mode, "frames_per_step": F, "parallelism": f"{args.mode}x{world}",
                "frames": ("one frame per rank and step: rank r renders frame r of the camera path through the "
                           "config's camera (scenes.rank_frame_spec; rank 0 the config's frame)")
                if args.mode == "frames" and F == 1 else
                ("rank r renders orbit frames r*F .. r*F+F-1 of the 256-frame C5 orbit in one launch"
                 if args.mode == "frames" else "one frame row-tiled over the ranks")},
            "roofline": {
                "bound": "valu",
                "kernel": f"k_render_fast<{B}>" if B is not None and B <= 6 else "k_render_fast<5, DEEP> (first pass)",
                "achieved": round(head_tflops, 4),
                "peak": PEAK_FP64_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(head_tflops / PEAK_FP64_TFLOPS, 5),
                "traffic": traffic,
                "kernel_ms": round(kern_avg_s * 1e3, 5),
                "kernel_launches_timed": kern_n,
                "flops_per_launch": head_flops,
                "flops_model": "executed (culling tree: tests the kernel ran)" if culled else "SURVEY.md 8d",
                "reference_equivalent": {
                    "achieved": round(achieved_tflops, 4), "frac": round(achieved_tflops / PEAK_FP64_TFLOPS, 5),
                    "flops_per_launch": flops,
                    "note": "the SURVEY.md 8d model: every ray tests all S spheres, as the reference does (culled "
                            "tests priced too: reference-equivalent throughput, not kernel efficiency)"},
                "executed_model": {
                    "achieved": round(achieved_exec, 4), "frac": round(achieved_exec / PEAK_FP64_TFLOPS, 5),
                    "flops_per_launch": flops_exec, "sphere_tests": st["sphere_tests"],
                    "node_tests": st["node_tests"], "box_tests": st["box_tests"],
                    "beam_tests": st["beam_tests"],
                    "sphere_tests_reference": S * (R_tr + R_sh),
                    "reflected_rays": {"sphere_tests": st["sphere_tests_reflected"],
                                       "node_tests": st["node_tests_reflected"],
                                       "beam_searches": st["beam_searches"], "beam_tests": st["beam_tests"],
                                       "wave_searches": sum(st["waves_traced"][1:])},
                    "note": "15/primary ray + 20/ray-sphere test + 22/culling-node test + 37/beam test + 200/shaded "
                            "hit over the tests k_render_fast executed (kernel counters); node_tests counts the "
                            "culling tree's box tests (box_tests) and, priced as node tests too, the shadow-grid "
                            "lookups; beam_tests the reflected-ray cone tests, one per live lane and beam pass (the "
                            "level-0 tile candidates' image-plane box comparisons are not priced); `achieved` above "
                            "prices every test the reference performs (S per ray), culled or not"},
                "lane_utilisation": {
                    "traced": [round(r / (64 * w), 4) if w else None for r, w in zip(st["rays"], st["waves_traced"])],
                    "shaded": [round(h / (64 * w), 4) if w else None for h, w in zip(st["hits"], st["waves_shaded"])],
                    "note": "live lanes / (64 x waves that ran the level), per level, fast kernel (the f3 "
                            "compaction question: wavefront compaction can only recover the idle lanes)"},
                "rays_per_level": st["rays"],
                "hits_per_level": st["hits"],
                "hbm": {"achieved": round(achieved_gbs, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(achieved_gbs / PEAK_HBM_GBS, 6), "alg_bytes_per_launch": alg_bytes},
                "note": "FP64 VALU-bound megakernel (no dense contraction, no MFMA); achieved = algorithmic "
                        "FLOPs (flops_model, kernel counters) / kernel time (HIP events on the launch "
                        f"stream around 1 in {every} launches of the timed region)",
            },
            "cpu_baseline": cpu,
            "output_path": out_path,
        }
        if secondary:
            line["secondary"] = secondary
            ss = strong_scaling(secondary, world)
            if ss:
                line["strong_scaling"] = ss
        if cpu:
            line["gpu_vs_cpu"] = round(value / cpu["value"], 1)
            if cpu.get("single_core"):
                line["gpu_vs_cpu_1core"] = round(value / cpu["single_core"]["value"], 1)
        s = json.dumps(line)
        print(s)
        if args.json_out:
            Path(args.json_out).write_text(s + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def frame_spec_for_rank(spec: dict, rank: int) -> dict:
    """The frame a rank renders in frames mode at one frame per step (tests/test_distributed_cpu.py
    checks, over a gloo world of 2, that the ranks' frames differ and rank 0's is the config's)."""
    from python_ray_tracer_amd import scenes

    return scenes.rank_frame_spec(spec, rank)


def tiles_stepper(r, scene, world, row_block, out, loopback=False, comm_reserve=None, rows=None, timed=False):
    """(step, drain) of the strong-scaling tiles mode: TileGather with two slots; step k submits
    frame k and finishes frame k-1 (its gather overlapped frame k's render); drain finishes the last
    one. Without a process group: the whole frame rendered into a pre-allocated buffer. ``timed``:
    the plan records its gathers (RTX_TILES_TIMED); ``step.timing()`` reads the last frame's."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():  # one process without a group: the whole frame, no gather
        W, H = int(scene.camera.width), int(scene.camera.height)
        buf = (torch.empty((H, W, 3), dtype=torch.uint8, device=r.device) if out == "u8"
               else torch.empty((3, W * H), dtype=r.color_dtype, device=r.device))

        def step1():
            return r.render_tile(scene, out=out, into=buf)
        return step1, (lambda: None)
    from python_ray_tracer_amd.distributed import TileGather

    tg = TileGather(r, int(scene.camera.width), int(scene.camera.height), row_block=row_block, out=out, slots=2,
                    persistent_frames=True, loopback=loopback, comm_reserve=comm_reserve, rows=rows, timed=timed)
    state = {"k": 0, "open": None, "last": None}

    def step():
        slot = state["k"] % 2
        tg.submit(scene, slot)
        if state["open"] is not None:
            tg.finish(state["open"])
        state["open"] = state["last"] = slot
        state["k"] += 1

    step.tg = tg
    step.timing = lambda: tg.timing(state["last"])

    def drain():
        if state["open"] is not None:
            tg.finish(state["open"])
            state["open"] = None
    return step, drain


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def secondary_tiles(args, r, scene, world, dev, coll_dev):
    """The strong-scaling row-tiled frame next to the headline, at every N:
    tiles mode — every rank renders its interleaved row tile into the gather buffer, the gather to
    rank 0, rtx_assemble_rows there, uint8 frame, two frames in flight (distributed.TileGather) — for
    the config and for C4 (7680x4320, the scaling config). At N=1 on a one-rank process group, so
    the N=1 point runs the same code as N>1. Timed like the headline (barrier, K steps, barrier,
    max over ranks); never fatal."""
    import torch
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    own_group = False
    try:
        if not dist.is_initialized():
            kw = {"device_id": dev} if args.backend == "nccl" else {}
            dist.init_process_group(args.backend, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                    world_size=1, **kw)
            own_group = True
    except Exception as e:  # noqa: BLE001 - a secondary measurement, never fatal
        return {"tiles_error": repr(e)[:300]}

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def timed(step, drain, k, warm):
        for _ in range(warm):
            step()
        drain()
        barrier()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        drain()
        barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    out = {}
    try:
        W, H = int(scene.camera.width), int(scene.camera.height)
        k = max(10, min(args.steps, 200))
        step, drain = tiles_stepper(r, scene, world, args.row_block, "u8")
        t = timed(step, drain, k, 5)
        out["tiles_u8"] = {"value": round(W * H * k / t / 1e6, 3), "unit": "Mpixels/s",
                           "ms_per_step": round(t / k * 1e3, 5), "steps": k, "scaling": "strong",
                           "config": f"{args.config} row-tiled over {world} rank(s) ({dist.get_backend()}): render "
                                     f"into the gather buffer (row_block {args.row_block}), gather to rank 0, "
                                     "rtx_assemble_rows, uint8 frame, two frames in flight"}
        c4spec, c4B = scenes.CONFIGS["C4"]()
        r4 = HipRenderer(max_bounces=c4B, color_dtype=torch.float32, device=dev,
                         learn_tile_order=not args.no_tile_order)
        # N = 1: a loopback plan (the tile still goes through RCCL, sent to and received from the
        # rank itself, then assembled), so that the one-GPU point runs the gather path of N > 1
        loop = world == 1 and dist.get_backend() == "nccl"
        step, drain = tiles_stepper(r4, scenes.build_scene(c4spec), world, args.row_block, "u8", loopback=loop,
                                    timed=dist.get_backend() == "nccl")
        k4 = 10
        t = timed(step, drain, k4, 2)
        out["c4_tiles"] = {"value": round(7680 * 4320 * k4 / t / 1e6, 3), "unit": "Mpixels/s",
                           "ms_per_step": round(t / k4 * 1e3, 5), "steps": k4, "scaling": "strong",
                           "config": "C4: 64 random spheres + ground 7680x4320 seed 0, 5 bounces, row-tiled over "
                                     f"{world} rank(s), gather of the uint8 frame to rank 0"
                                     + (" (one-rank loopback plan: the tile sent to and received from the rank "
                                        "itself over RCCL, then assembled)" if loop else "")}
        if getattr(getattr(step, "tg", None), "timed", False):
            out["c4_tiles"]["gather"] = gather_timing(step.timing(), world, loop)
        # the strong-scaling speed-up in the same run: rank 0 alone renders the whole C4 frame
        # as the one-rank tiles path does (straight into the uint8 frame), the others wait (at
        # N = 1 the ratio is the loopback plan's overhead over the plain frame)
        if dist.get_rank() == 0:
            c4 = scenes.build_scene(c4spec)
            buf = torch.empty((4320, 7680, 3), dtype=torch.uint8, device=dev)
            for _ in range(2):
                r4.render_tile(c4, out="u8", into=buf)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(k4):
                r4.render_tile(c4, out="u8", into=buf)
            torch.cuda.synchronize(dev)
            t1 = (time.perf_counter() - t0) / k4
            out["c4_tiles"]["single_gpu_ms_per_step"] = round(t1 * 1e3, 5)
            out["c4_tiles"]["speedup_vs_1gpu"] = round(t1 / (t / k4), 4)
        dist.barrier()
    except Exception as e:  # noqa: BLE001
        if world > 1:
            # N > 1: the row-tiled frame is the north star's multi-GPU mechanism; a broken plan must
            # fail the run (non-zero exit), not hide behind a green headline
            raise
        out["tiles_error"] = repr(e)[:300]
    finally:
        if own_group:
            dist.destroy_process_group()
    return out


def gather_timing(mine: dict, world: int, loop: bool) -> dict:
    """The C4 tiles leg's measured gather (rtx_tiles_timing on every rank, last timed frame):
    bytes per peer, the root's span (its tile rendered -> every part received) and its assembly,
    each peer's send span (its tile rendered -> delivered; the root's receive is posted when the
    root's smaller share has rendered), and the achieved rate per link = part bytes / send span."""
    import torch.distributed as dist

    allt = [mine]
    if world > 1:
        allt = [None] * world
        dist.all_gather_object(allt, mine)
    root = allt[0]
    g = {"part_bytes": root["part_bytes"], "root_gather_ms": round(root["gather_ms"], 4),
         "root_assemble_ms": round(root["assemble_ms"], 4), "root_received_bytes": root["bytes"]}
    if loop:
        # HBM to HBM on one GPU: never an xGMI figure
        g["link"] = "loopback (HBM)"
        g["loopback_GBps"] = round(root["part_bytes"] / max(root["gather_ms"], 1e-6) / 1e6, 2)
        g["xgmi_GBps_per_peer"] = None
    else:
        peers = [a["gather_ms"] for a in allt[1:]]
        g["link"] = "xGMI point-to-point, one peer per link into the root"
        g["peer_send_ms"] = [round(x, 4) for x in peers]
        g["xgmi_GBps_per_peer"] = [round(root["part_bytes"] / max(x, 1e-6) / 1e6, 2) for x in peers]
        g["xgmi_GBps_min"] = min(g["xgmi_GBps_per_peer"]) if peers else None
        g["root_in_GBps"] = round(root["bytes"] / max(root["gather_ms"], 1e-6) / 1e6, 2)
    return g


# The xGMI rate DESIGN.md §6's 1 -> 8 prediction assumes for RCCL point-to-point traffic (per link and
# direction). The one place it lives: a bench line that measured the gather over xGMI reports the
# measured rate beside it (strong_scaling.gather.xgmi_GBps_min), which replaces it.
ASSUMED_XGMI_GBPS = 40.0


def strong_scaling(secondary: dict | None, world: int) -> dict | None:
    """The row-tiled C4 frame (the north star's multi-GPU mechanism) at the top level of the line:
    its throughput, the whole frame rendered by rank 0 alone in the same run, the speed-up, and the
    gather per peer (bytes, ms, GB/s per link). From ``secondary.c4_tiles``; None without it."""
    c4 = (secondary or {}).get("c4_tiles")
    if not c4:
        return None
    out = {"config": c4["config"], "n_gpus": world, "value": c4["value"], "unit": c4["unit"],
           "ms_per_step": c4["ms_per_step"], "single_gpu_ms_per_step": c4.get("single_gpu_ms_per_step"),
           "speedup_vs_1gpu": c4.get("speedup_vs_1gpu"),
           "note": "speedup_vs_1gpu = rank 0 rendering the whole C4 frame alone / the row-tiled frame over "
                   "n_gpus ranks with its RCCL gather, both in this run (N = 1: a loopback plan, the "
                   "ratio is the gather path's overhead)"}
    g = c4.get("gather")
    if g:
        out["gather"] = g
        measured = g.get("xgmi_GBps_min")
        out["xgmi_GBps"] = {"measured": measured, "assumed": None if measured else ASSUMED_XGMI_GBPS,
                            "note": "DESIGN.md §6 predicts the 1 -> 8 curve from the assumed rate until a "
                                    "run over xGMI measures it"}
    return out


def emulate_parts(args, r, scene, spec, B, part_counts):
    """The compute side of the N-GPU row-tiled frame on one GPU: for each N,
    every part p of render_tile(scene, row_block, N, p) is rendered into its slot of an [N,
    part_len] uint8 gather buffer, as rank p would, and timed — the fast kernel by the library's HIP
    events, the whole launch (fast + general kernel, host call) by wall clock over K synchronised
    launches — then rtx_assemble_rows of the N parts (the root's un-permute), whose frame must equal
    the single-GPU render. Each rank's share follows the plan's (--shares, else
    distributed.ROOT_SHARES): the root renders root_run parts, every other rank run parts of the
    root_run + (N-1)*run interleave. The gather itself is not emulated: DESIGN.md §6 prices it from
    the part bytes reported here."""
    import numpy as np
    import torch

    from python_ray_tracer_amd import tiling
    from python_ray_tracer_amd.infrastructure.hip import _lib as L

    W, H = int(scene.camera.width), int(scene.camera.height)
    dev = r.device
    rb = args.row_block
    k = max(5, min(args.steps, 100))

    def kernel_us(fn):
        fn()
        torch.cuda.synchronize(dev)
        L.profile_sample(1)
        L.profile_enable(k)
        for _ in range(k):
            fn()
        ms, n = L.profile_collect()
        L.profile_enable(0)
        return ms / max(n, 1) * 1e3

    def wall_us(fn):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / k * 1e6

    whole = r.render_tile(scene, out="u8")
    from python_ray_tracer_amd.distributed import ROOT_SHARES

    res = {}
    for N in sorted({1, *part_counts}):
        root_run, run = ((int(v) for v in args.shares.split(",")) if args.shares and N > 1
                         else ROOT_SHARES.get(N, (1, 1)))
        n_parts, shares = tiling.runs(N, root_run, run)
        plen = tiling.part_len(H, W, rb, N, 1, "u8", root_run, run)
        tiles = torch.zeros((N, plen), dtype=torch.uint8, device=dev)
        parts = []
        for p, (first, k_run) in enumerate(shares):
            shp = tiling.tile_shape(H, W, rb, n_parts, first, "u8", k_run)
            view = tiles[p, :int(np.prod(shp))].view(shp)

            def fn(first=first, k_run=k_run, view=view):
                return r.render_tile(scene, rb, n_parts, first, out="u8", into=view, part_run=k_run)
            parts.append({"rank": p, "parts": [first, k_run], "rows": shp[0], "kernel_us": round(kernel_us(fn), 3),
                          "launch_us": round(wall_us(fn), 3)})
        frame = r.assemble_rows(tiles, W, H, rb, "u8", root_run, run)
        if not torch.equal(frame, whole):
            raise AssertionError(f"assembled {N}-rank frame differs from the whole-frame render")
        asm_us = wall_us(lambda: r.assemble_rows(tiles, W, H, rb, "u8", root_run, run))
        kus = [q["kernel_us"] for q in parts]
        lus = [q["launch_us"] for q in parts]
        res[str(N)] = {"shares": [root_run, run], "kernel_us_max": max(kus), "kernel_us_mean": round(sum(kus) / N, 3),
                       "root_kernel_us": kus[0], "peer_kernel_us_max": max(kus[1:]) if N > 1 else None,
                       "imbalance": round(max(kus) / (sum(kus) / N), 4), "launch_us_max": max(lus),
                       "assemble_us": round(asm_us, 3), "part_bytes": plen, "root_receives_bytes": (N - 1) * plen,
                       "frame_equals_single_gpu": True, "parts": parts}
    return {"metric": "per-part row-tile render time, 1-GPU emulation of the N-GPU frame", "unit": "us",
            "config": {"workload": args.config, "width": W, "height": H, "max_bounces": B,
                       "spheres": len(spec["spheres"]), "row_block": rb, "output": "u8", "launches_per_part": k},
            "n": res,
            "note": "kernel_us: k_render_fast by HIP events (library); launch_us: one render_tile call end to end "
                    "(fast + general kernel and the host call), K synchronised calls; assemble_us: "
                    "rtx_assemble_rows of the N parts on the root"}


def cpu_baseline_or_error(spec, B, procs, budget_s, single, timeout_s=None):
    """cpu_baseline_all_cores, or the 1-core baseline with ``all_cores_error`` when the all-cores
    leg fails or times out: the baseline is reported, never fatal."""
    try:
        return cpu_baseline_all_cores(spec, B, procs, budget_s, single, timeout_s)
    except Exception as e:  # noqa: BLE001
        out = dict(single)
        out["all_cores_error"] = repr(e)[:300]
        return out


def cpu_baseline_all_cores(spec, B, procs, budget_s, single, timeout_s=None):
    """The oracle row-tiled over ``procs`` processes (one core each) through the gloo multi-rank
    path (oracle/row_tiled.py): render + gather of whole frames (frames up to 2.5 Mpixels) or of
    a sample of interleaved row tiles (C3, C4). ``single``: the 1-core result, kept beside it.
    Runs in a child process group killed after ``timeout_s`` (raises TimeoutError)."""
    import math

    from oracle import row_tiled

    procs = max(1, min(procs, row_tiled.host_cores()))
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    sub = 1 if W * H <= 2_500_000 else math.ceil(W * H / (procs * 600_000))
    t_step = W * H / sub / (single["value"] * 1e6) / procs * 1.3  # estimated wall time of one step
    frames = int(max(2, min(20, budget_s / max(t_step, 1e-3))))
    # in a child process group with a hard limit: a stuck gloo rendezvous cannot hold the JSON line
    # back (start-up and imports of the workers take ~10-20 s on a fresh box)
    limit = timeout_s if timeout_s is not None else 90.0 + 3.0 * frames * t_step
    res = row_tiled.run_bounded(spec, B, procs, frames, sub, limit)
    rate = max(p / t for p, t in zip(res["pixels"], res["times"]))
    what = (f"{frames} full {W}x{H} frames" if sub == 1 else
            f"{frames} samples of {procs} interleaved row tiles (1/{sub} of the {W}x{H} frame each)")
    return {"value": round(rate / 1e6, 4), "unit": "Mpixels/s", "cores": procs, "kind": "port",
            "sample": f"{what}, B={B}, oracle/numpy_oracle.py row-tiled over {procs} processes "
                      f"(oracle/row_tiled.py, gloo gather to rank 0), best step of {frames} "
                      f"(median {sorted(res['times'])[len(res['times']) // 2]:.3f}s)",
            "single_core": single}


def output_path_times(r, scene):
    """save_image's work for one frame, outside the timed step: device quantisation
    to uint8 [H, W, 3], the D2H copy, and the PNG encode (best of 3 each)."""
    import io

    import torch

    from python_ray_tracer_amd.infrastructure.hip.base import _write_png

    color = r.render(scene)
    q, d2h, png = [], [], []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        u8 = r.quantize(color, scene.camera)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        host = u8.cpu().numpy()
        t2 = time.perf_counter()
        _write_png(host, io.BytesIO())
        t3 = time.perf_counter()
        q.append(t1 - t0)
        d2h.append(t2 - t1)
        png.append(t3 - t2)
    return {"quantize_ms": round(min(q) * 1e3, 4), "d2h_ms": round(min(d2h) * 1e3, 4),
            "png_encode_ms": round(min(png) * 1e3, 3), "bytes": int(host.nbytes),
            "note": "not in the timed step; PNG encode is PIL on one host core (base.py:143-151)"}


def cpu_baseline(spec, B, budget_s):
    """The CPU oracle (NumPy float64, the reference's algorithm; single process => 1 core) on the
    same configuration until ``budget_s`` seconds of CPU work: whole frames up to 2.5 Mpixels
    (best frame), otherwise interleaved row tiles of ~0.5 Mpixels spread over the frame (total
    pixels / total time). Ray generation + trace, no PNG — the same region as a GPU step."""
    import math
    import platform

    from oracle import numpy_oracle as O
    from python_ray_tracer_amd import tiling

    sc = O.scene_from_spec(spec)
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    parts = 1 if W * H <= 2_500_000 else math.ceil(W * H / 500_000)
    times, pixels = [], []
    t_start = time.perf_counter()
    k = 0
    while True:
        t0 = time.perf_counter()
        if parts == 1:
            O.render(sc, B)
            pixels.append(W * H)
        else:
            part = (k * 7919) % parts  # spread over the frame (sky and ground rows alike)
            rows = tiling.tile_rows(H, 8, parts, part)
            O.render_rows(sc, rows, B)
            pixels.append(W * len(rows))
        times.append(time.perf_counter() - t0)
        k += 1
        if time.perf_counter() - t_start >= budget_s or len(times) >= 50:
            break
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    if parts == 1:
        value = W * H / min(times)
        what = f"{len(times)} full {W}x{H} frames, B={B}, best of {len(times)} (median {sorted(times)[len(times) // 2]:.3f}s)"
    else:
        value = sum(pixels) / sum(times)
        what = (f"{len(times)} interleaved row tiles (1/{parts} of the {W}x{H} frame each, row blocks of 8), B={B}, "
                f"{sum(pixels)} pixels in {sum(times):.1f}s")
    return {"value": round(value / 1e6, 4), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"{what}; oracle/numpy_oracle.py, {cpu_model or platform.processor()}"}


if __name__ == "__main__":
    main()
