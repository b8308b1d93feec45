"""The round-5 capture crash (session r5a) re-run in isolation: a gathering native tiles plan (a
one-rank loopback plan: render, RCCL send/receive to itself, assembly) captured into a HIP graph the
way tests/test_gpu_distributed.py did at commit dd6da5d, with a native backtrace on a fatal signal
(tools/libsegv_trace.so). TileGather refuses to submit a gathering plan under capture since round 5;
this script drives the plan's own entry point (HipRenderer.submit_tiles, what TileGather.submit
calls) to reach the capture anyway.

    python tools/capture_tiles.py VARIANT        (VARIANT: assembled | rows | fresh | ops_torch | ops_raw)

``fresh``: the captured frame goes through a second plan whose slot has carried no frame, so
rtx_tiles_submit does not wait on the slot's `done` event recorded before the capture began.
``ops_torch`` / ``ops_raw``: no torch.distributed process group at all (no ProcessGroupNCCL
communicator in the process): the loopback plan is made through the torch ops (rt::comm_init,
rt::tiles_create) and captured by torch.cuda.graph, or by hipStreamBeginCapture/EndCapture called
directly (ctypes on the process's libamdhip64).

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


def ops_variant(variant):
    """A loopback plan through the torch ops, no process group; captured by torch or by raw HIP."""
    import torch

    import python_ray_tracer_amd.ops  # noqa: F401
    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dev = torch.cuda.current_device()
    W, H, B = 96, 61, 3
    sc = scenes.build_scene(scenes.random_spec(40, 6, W, H))
    r = HipRenderer(max_bounces=B, color_dtype=torch.float32)
    want = r.render_tile(sc, out="u8").clone()
    blob, S = r.scene_blob(sc)
    ws = torch.zeros(torch.ops.rt.workspace_bytes(W * H, B), dtype=torch.uint8, device="cuda")
    part = (W * H * 3 + 15) // 16 * 16
    comm = torch.ops.rt.comm_init(torch.ops.rt.comm_unique_id(), 1, 0, dev)
    send = [torch.zeros(part, dtype=torch.uint8, device="cuda")]
    recv = [torch.zeros(part, dtype=torch.uint8, device="cuda")]
    plan = torch.ops.rt.tiles_create(comm, 1, 0, 0, W, H, 8, 2, 1, send, recv, part, flags=1, device=dev)
    frame = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    torch.ops.rt.tiles_submit(plan, 0, blob, S, B, ws, frame)
    torch.ops.rt.tiles_finish(plan, 0, dev)
    torch.cuda.synchronize()
    say(f"eager frame {'equal' if torch.equal(frame, want) else 'DIFFERS'} (ops, no process group)")
    trace = REPO / "tools" / "libsegv_trace.so"
    if trace.exists():
        ctypes.CDLL(str(trace)).segv_trace_install()
        say("segv trace handler installed")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    if variant == "ops_torch":
        g = torch.cuda.CUDAGraph()
        say("capture begin (torch.cuda.graph)")
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            torch.ops.rt.tiles_submit(plan, 0, blob, S, B, ws, frame)
            torch.ops.rt.tiles_finish(plan, 0, dev)
            say("  submitted and finished; capture_end next")
        say("capture end")
        replay = g.replay
    else:
        import os

        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))  # torch's (loaded)
        graph, exe = ctypes.c_void_p(), ctypes.c_void_p()
        sh = ctypes.c_void_p(s.cuda_stream)
        say("capture begin (hipStreamBeginCapture, global mode)")
        assert hip.hipStreamBeginCapture(sh, 0) == 0
        with torch.cuda.stream(s):
            torch.ops.rt.tiles_submit(plan, 0, blob, S, B, ws, frame)
            torch.ops.rt.tiles_finish(plan, 0, dev)
        say("  submitted and finished; hipStreamEndCapture next")
        rc = hip.hipStreamEndCapture(sh, ctypes.byref(graph))
        say(f"hipStreamEndCapture rc={rc}")
        assert rc == 0
        assert hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, ctypes.c_size_t(0)) == 0
        say("instantiated")

        def replay():
            assert hip.hipGraphLaunch(exe, sh) == 0
    for k in range(3):
        frame.zero_()
        torch.cuda.synchronize()
        replay()
        torch.cuda.synchronize()
        say(f"replay {k}: {'equal' if torch.equal(frame, want) else 'MISMATCH'}")
    torch.ops.rt.tiles_destroy(plan)
    torch.ops.rt.comm_destroy(comm)
    say("ok")


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "assembled"
    if variant.startswith("ops_"):
        return ops_variant(variant)
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
