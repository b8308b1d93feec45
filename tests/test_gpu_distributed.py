"""The multi-rank render path with HipRenderer tiles on the GPU.

The box has one GPU and RCCL needs one GPU per rank, so two fresh torchrun ranks share the GPU
over gloo (tiles travel through host memory; on an 8-GPU node the same code runs over RCCL). The
frame they gather and assemble on the device must equal the single-rank frame bit for bit — colour
and uint8 gathers, capped and unbounded bounces, a 65-sphere scene — and render_image_pipeline's
PNG must equal the single-rank pipeline's. Also the two-slot pipelined gather (bench --mode tiles).
"""

import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_share_gpu_gather_equals_single_frame(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "tests" / "dist_hip_worker.py"),
           str(tmp_path)]
    p = subprocess.run(cmd, cwd=str(REPO), env=env, capture_output=True, text=True, timeout=110)
    logs = {f.name: f.read_text() for f in tmp_path.glob("rank*.txt")}
    assert p.returncode == 0, (p.returncode, logs, p.stdout[-3000:], p.stderr[-3000:])
    assert set(logs) == {"rank0.txt", "rank1.txt"}, logs
    assert "False" not in logs["rank0.txt"] and "png_u8" in logs["rank0.txt"], logs


def test_native_tiles_world_gt1_through_rccl_stub():
    """The native plan's world > 1 code (rtx_tiles.hip: the root's per-peer receives into
    recv + p * part_bytes while it renders its own share, the peers' sends, rtx_assemble_runs over
    the weighted shares 8:9 / 3:4 / 1:2, gather_rows for RTX_TILES_ROWS) on the box's one GPU: N ranks
    as threads of one fresh process, each with its own renderer, stream and plan, RCCL bound to the
    test-only stub (tests/stub_rccl.cpp: sends matched to receives in posting order, device copies on
    the receiver's stream). Two slots in flight; u8 and f32; capped and unbounded. The root's frames
    equal the single-GPU render bit for bit and the stub's log holds exactly the operations the plan's
    layout implies (tests/stub_tiles_worker.py)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json

    stub = REPO / "tests" / "libstub_rccl.so"
    if not stub.exists():  # build() warns and goes on when the test-only stand-in fails to compile
        pytest.skip("tests/libstub_rccl.so not built (see build()'s warning)")
    p = subprocess.run([sys.executable, "-u", str(REPO / "tests" / "stub_tiles_worker.py")], cwd=str(REPO),
                       capture_output=True, text=True, timeout=115)
    lines = [json.loads(s) for s in p.stdout.splitlines() if s.startswith("{")]
    assert p.returncode == 0, (p.returncode, lines, p.stderr[-3000:])
    cases = {c["case"]: c for c in lines if "case" in c}
    assert {"n2_8to9_f32", "n4_3to4_u8", "n8_1to2_u8", "n8_1to2_f32", "n4_rows_u8",
            "n3_3to4_f32_unbounded"} <= set(cases), cases
    for c in cases.values():
        assert c["ok"] and all(c["frames_equal"]) and c["log_matches"], c


def test_nccl_two_slot_pipeline_equals_single_frames():
    """TileGather under nccl (a one-rank RCCL group on the box's one GPU): orbit frames pushed
    through the two-slot pipeline of bench.py's tiles mode (submit k, finish k-1; the gather runs on
    RCCL's stream), capped and unbounded, colour and uint8, equal the single-GPU frames bit for bit;
    so does the synchronous one-slot path."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.distributed import TileGather
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        base = scenes.random_spec(16, 5, 96, 61)
        frames = [scenes.build_scene(scenes.with_camera(base, scenes.orbit_position(k, 12))) for k in range(6)]
        for B, out in ((3, "u8"), (None, None)):
            r = HipRenderer(max_bounces=B, color_dtype=torch.float32, device=dev)
            want = [r.render_tile(sc, out=out).clone() for sc in frames]
            tg = TileGather(r, 96, 61, row_block=4, out=out, slots=2)
            got, open_slot = [], None
            for k, sc in enumerate(frames):
                tg.submit(sc, k % 2)
                if open_slot is not None:
                    got.append(tg.finish(open_slot))
                open_slot = k % 2
            got.append(tg.finish(open_slot))
            torch.cuda.synchronize()
            for k in range(len(frames)):
                assert torch.equal(got[k], want[k]), (B, k)
            one = TileGather(r, 96, 61, row_block=4, out=out, slots=1)
            assert torch.equal(one.render(frames[2]), want[2])
    finally:
        dist.destroy_process_group()


def test_native_tiles_loopback_and_graph_replay():
    """The native row-tiled step (rtx_tiles_submit) on a one-rank RCCL group: (1) a loopback plan —
    the tile sent to and received from the rank itself over RCCL, row block by row block straight
    into the frame (RTX_TILES_ROWS) or whole and then assembled — gives the single-GPU frames bit
    for bit through the two-slot pipeline; (2) a render_tile(into=) frame and
    a native tiles step captured into HIP graphs (include/rtx_hip.h: the entry points never
    allocate or synchronise) replay to the eager frames bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.distributed import TileGather
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        base = scenes.random_spec(40, 2, 104, 57)
        frames = [scenes.build_scene(scenes.with_camera(base, scenes.orbit_position(k, 9))) for k in range(5)]
        r = HipRenderer(max_bounces=4, color_dtype=torch.float32, device=dev)
        want = [r.render_tile(sc, out="u8").clone() for sc in frames]
        for rows in (True, False):  # row blocks straight into the frame (RTX_TILES_ROWS), or assembled
            tg = TileGather(r, 104, 57, row_block=8, out="u8", slots=2, loopback=True, rows=rows)
            assert tg.plan is not None and tg.send and tg.recv is not None and tg.rows == rows
            got, open_slot = [], None
            for k, sc in enumerate(frames):
                tg.submit(sc, k % 2)
                if open_slot is not None:
                    got.append(tg.finish(open_slot))
                open_slot = k % 2
            got.append(tg.finish(open_slot))
            torch.cuda.synchronize()
            for k in range(len(frames)):
                assert torch.equal(got[k], want[k]), (rows, k)

        sc = frames[3]
        buf = torch.empty_like(want[3])
        r.render_tile(sc, out="u8", into=buf)  # eager first: code objects, scene upload, workspace
        tgd = TileGather(r, 104, 57, row_block=8, out="u8", slots=1, persistent_frames=True)
        torch.cuda.synchronize()
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            r.render_tile(sc, out="u8", into=buf)
        with torch.cuda.graph(g2):
            tgd.submit(sc, 0)
            tgd.finish(0)
        for _ in range(2):
            buf.zero_()
            tgd.frames[0].zero_()
            g1.replay()
            g2.replay()
            torch.cuda.synchronize()
            assert torch.equal(buf, want[3])
            assert torch.equal(tgd.frames[0], want[3])
        # the pins a capture takes are keyed by address: capturing the same launch again pins nothing
        # new (a long-lived renderer recapturing graphs must not grow without bound)
        npins = len(r._graph_pins)
        assert npins >= 2
        g3 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g3):
            r.render_tile(sc, out="u8", into=buf)
        assert len(r._graph_pins) == npins
        del g1, g2, g3
        assert r.release_graph_pins() == npins and not r._graph_pins
    finally:
        dist.destroy_process_group()


def test_gathering_plan_refuses_graph_capture(monkeypatch):
    """RCCL send/recv captured into a HIP graph crashes the end of the capture in this image (a stack
    overflow in torch's bundled HIP runtime's hipStreamEndCapture, triggered by the RCCL group:
    DESIGN.md §6, tools/capture_tiles.py), so TileGather refuses to submit a gathering plan under
    stream capture with a RuntimeError instead; a one-rank plan without RCCL traffic still captures
    (test_native_tiles_loopback_and_graph_replay)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.distributed import TileGather
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        sc = scenes.build_scene(scenes.random_spec(40, 6, 96, 61))
        r = HipRenderer(max_bounces=3, color_dtype=torch.float32, device=dev)
        want = r.render_tile(sc, out="u8").clone()
        tg = TileGather(r, 96, 61, row_block=8, out="u8", slots=1, loopback=True, persistent_frames=True)
        monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
        with pytest.raises(RuntimeError, match="cannot be captured"):
            tg.submit(sc, 0)
        monkeypatch.undo()
        tg.submit(sc, 0)  # eagerly: fine
        assert torch.equal(tg.finish(0), want)
    finally:
        dist.destroy_process_group()
