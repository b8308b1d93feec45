"""The round-5 capture crash (session r5a) re-run in isolation: a gathering native tiles plan (a
one-rank loopback plan: render, RCCL send/receive to itself, assembly) captured into a HIP graph the
way tests/test_gpu_distributed.py did at commit dd6da5d, with a native backtrace on a fatal signal
(tools/libsegv_trace.so). TileGather refuses to submit a gathering plan under capture since round 5;
this script drives the plan's own entry point (HipRenderer.submit_tiles, what TileGather.submit
calls) to reach the capture anyway.

    python tools/capture_tiles.py VARIANT        (VARIANT: assembled | rows | fresh)

``fresh``: the captured frame goes through a second plan whose slot has carried no frame, so
rtx_tiles_submit does not wait on the slot's `done` event recorded before the capture began.

Prints one line per step, then "ok" with the replays' result; exits 139 with the backtrace on a
segmentation fault. Run it in its own process (tools/session.sh capture:VARIANT).
"""

from __future__ import annotations

import ctypes
import socket
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def say(*a):
    print(*a, flush=True)


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "assembled"
    import torch
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.distributed import TileGather
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dev = torch.device("cuda", 0)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    sc = scenes.build_scene(scenes.random_spec(40, 6, 96, 61))
    r = HipRenderer(max_bounces=3, color_dtype=torch.float32, device=dev)
    want = r.render_tile(sc, out="u8").clone()
    tg = TileGather(r, 96, 61, row_block=8, out="u8", slots=1, loopback=True, rows=(variant == "rows"),
                    persistent_frames=True)
    tg.submit(sc, 0)  # eager first: the learnt order, the probe, RCCL's own set-up
    assert torch.equal(tg.finish(0), want)
    torch.cuda.synchronize()
    say("eager frame equal")

    if variant == "fresh":  # a plan whose slot has never been used: no wait on a pre-capture event
        tg = TileGather(r, 96, 61, row_block=8, out="u8", slots=1, loopback=True, persistent_frames=True)
        say("fresh plan for the capture")

    def submit_captured():  # TileGather.submit's plan branch, without its capture guard
        frame = tg.frames[0]
        r.submit_tiles(tg.plan, 0, sc, tg.rb, tg.n_parts, tg.first, frame, part_run=tg.my_run)
        tg._pending[0] = (None, frame)

    trace = REPO / "tools" / "libsegv_trace.so"
    if trace.exists():  # after torch's own handlers: ours names the native frames of a crash
        ctypes.CDLL(str(trace)).segv_trace_install()
        say("segv trace handler installed")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    say("capture begin")
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            submit_captured()
            say("  submitted inside the capture")
            tg.finish(0)
            say("  finished inside the capture; capture_end next")
    say("capture end")
    torch.cuda.synchronize()
    for k in range(3):
        tg.frames[0].zero_()
        g.replay()
        torch.cuda.synchronize()
        say(f"replay {k}: {'equal' if torch.equal(tg.frames[0], want) else 'MISMATCH'}")
    dist.destroy_process_group()
    say("ok")


if __name__ == "__main__":
    main()
