"""The multi-rank paths of application.py on CPU: world_size 2 (and 3) processes over gloo.

The per-rank tile renderer here is a stand-in built on the CPU oracle (tests may use the oracle);
on the GPU box the same code runs with HipRenderer.render_tile and the nccl (RCCL) backend.
"""

import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pathlib import Path

from oracle import numpy_oracle as O
from python_ray_tracer_amd import scenes, tiling
from python_ray_tracer_amd.application import render_frame_distributed, render_frames
from python_ray_tracer_amd.distributed import TileGather


REPO = Path(__file__).resolve().parent.parent


class OracleTileRenderer:
    """render_tile contract of HipRenderer, computed by the oracle (CPU tensors)."""

    def __init__(self, B):
        self.B = B

    def render_tile(self, scene, row_block, n_parts, part, out=None, part_run=1):
        sc = O.scene_from_objects(scene)
        W, H = sc.width, sc.height
        rows = tiling.tile_rows(H, row_block, n_parts, part, part_run)
        full = O.render(sc, self.B).reshape(3, H, W)
        t = full[:, rows].reshape(3, -1)
        if out == "u8":
            return torch.from_numpy(O.to_uint8(t, W, len(rows)).copy())
        return torch.from_numpy(np.ascontiguousarray(t))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, spec, B, row_block, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = scenes.build_scene(spec)
        r = OracleTileRenderer(B)
        frame = render_frame_distributed(scene, r, row_block=row_block)
        frame_u8 = render_frame_distributed(scene, r, row_block=row_block, gather="u8")
        # two frames in flight through the pipelined gather (bench.py --mode tiles)
        orbit = scenes.build_scene(scenes.with_camera(spec, scenes.orbit_position(3, 8)))
        tg = TileGather(r, spec["camera"]["width"], spec["camera"]["height"], row_block=row_block, slots=2)
        tg.submit(scene, 0)
        tg.submit(orbit, 1)
        f0, f1 = tg.finish(0), tg.finish(1)
        # rows=True (RTX_TILES_ROWS on a native plan) takes even shares: the native plan moves parts
        # of one run each; explicit unequal shares with rows are refused up front
        W, H = spec["camera"]["width"], spec["camera"]["height"]
        tgr = TileGather(r, W, H, row_block=row_block, out="u8", rows=True)
        assert (tgr.root_run, tgr.run) == (1, 1)
        f_rows = tgr.render(scene)
        try:
            TileGather(r, W, H, row_block=row_block, out="u8", rows=True, shares=(1, 2))
        except ValueError:
            pass
        else:
            raise AssertionError("unequal shares with rows=True must be refused")
        if rank == 0:
            np.save(os.path.join(outdir, "rows_u8.npy"), f_rows.numpy())
            np.save(os.path.join(outdir, "frame.npy"), frame.numpy())
            np.save(os.path.join(outdir, "frame_u8.npy"), frame_u8.numpy())
            np.save(os.path.join(outdir, "pipe0.npy"), f0.numpy())
            np.save(os.path.join(outdir, "pipe1.npy"), f1.numpy())
        else:
            assert frame is None and frame_u8 is None and f0 is None and f1 is None
        # the synchronous path's cached TileGathers: one slot each, at most TILE_GATHER_CACHE kept
        from python_ray_tracer_amd.distributed import TILE_GATHER_CACHE

        cache = r._tile_gathers
        assert len(cache) == 2 and all(len(t.send) == 1 for t in cache.values())
        for w in range(TILE_GATHER_CACHE + 1):
            small = scenes.build_scene(scenes.readme_spec(8 + w, 5))
            f = render_frame_distributed(small, r, row_block=row_block)
            if rank == 0:
                assert np.array_equal(f.numpy(), O.render(O.scene_from_spec(scenes.readme_spec(8 + w, 5)), B))
        assert len(cache) == TILE_GATHER_CACHE

        # animation driver: frames sharded round-robin, no collective
        class FrameRenderer:
            def render(self, sc):
                return sc.camera.position.x

        got = render_frames([scenes.build_scene(scenes.with_camera(spec, scenes.orbit_position(k, 8)))
                             for k in range(8)], FrameRenderer())
        np.save(os.path.join(outdir, f"frames_{rank}.npy"), np.array(sorted(got)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,row_block", [(2, 8), (3, 4), (4, 4)])
def test_row_tiles_gather_equals_single_frame(world, row_block):
    """The default shares (ROOT_SHARES): the root renders fewer row blocks than a peer; on this
    27-row frame world 2 leaves the peer no rows and world 3 the last rank none (empty tiles)."""
    spec = scenes.readme_spec(40, 27)  # 27 rows: uneven split, padding exercised
    B = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), spec, B, row_block, d), nprocs=world,
                           start_method="spawn", join=True)
        frame = np.load(os.path.join(d, "frame.npy"))
        frame_u8 = np.load(os.path.join(d, "frame_u8.npy"))
        want = O.render(O.scene_from_spec(spec), B)
        assert np.array_equal(frame, want)
        assert np.array_equal(frame_u8, O.to_uint8(want, 40, 27))
        assert np.array_equal(np.load(os.path.join(d, "rows_u8.npy")), O.to_uint8(want, 40, 27))
        assert np.array_equal(np.load(os.path.join(d, "pipe0.npy")), want)
        orbit = O.render(O.scene_from_spec(scenes.with_camera(spec, scenes.orbit_position(3, 8))), B)
        assert np.array_equal(np.load(os.path.join(d, "pipe1.npy")), orbit)
        shards = [set(np.load(os.path.join(d, f"frames_{r}.npy")).tolist()) for r in range(world)]
        assert set().union(*shards) == set(range(8))
        for r in range(world):
            assert shards[r] == {k for k in range(8) if k % world == r}


def _headline_worker(rank, world, port, outdir):
    """One rank of the bench headline at N = world (frames mode, one frame per step): the frame
    bench.py picks for this rank, rendered by the oracle at a small size, its hash gathered."""
    import hashlib
    import sys

    sys.path.insert(0, str(REPO))
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec, B = scenes.CONFIGS["C2"]()
        small = scenes.with_camera(spec, width=48, height=27)
        mine = bench.frame_spec_for_rank(small, rank)
        img = O.render(O.scene_from_spec(mine), B)
        got = [None] * world
        dist.all_gather_object(got, (mine["camera"]["position"], hashlib.sha256(img.tobytes()).hexdigest()))
        if rank == 0:
            np.save(os.path.join(outdir, "rank0.npy"), img)
            with open(os.path.join(outdir, "ranks.txt"), "w") as f:
                f.write(repr(got))
    finally:
        dist.destroy_process_group()


def test_headline_ranks_render_distinct_frames():
    """at N > 1 the frames-mode headline renders a different frame on every rank
    (frame r of the camera path through the config's camera), and rank 0's frame is the N = 1
    line's (the config's own frame), so SCALE's N = 1 point equals BENCH."""
    import ast

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_headline_worker, args=(world, _free_port(), d), nprocs=world, start_method="spawn",
                           join=True)
        got = ast.literal_eval(open(os.path.join(d, "ranks.txt")).read())
        spec, B = scenes.CONFIGS["C2"]()
        small = scenes.with_camera(spec, width=48, height=27)
        assert got[0][0] == small["camera"]["position"]
        assert got[0][0] != got[1][0] and got[0][1] != got[1][1]  # distinct cameras and images
        assert np.array_equal(np.load(os.path.join(d, "rank0.npy")), O.render(O.scene_from_spec(small), B))
    # the path stays in front of the reference's fixed screen (z < 0) for all 256 frames
    assert all(scenes.path_position(spec, k)[2] <= spec["camera"]["position"][2] for k in range(256))


def test_default_shares():
    """TileGather's default shares: ROOT_SHARES with the root at rank 0, even shares for a root
    elsewhere and for row-block gathers (RTX_TILES_ROWS takes runs of one part: ADVICE r4)."""
    from python_ray_tracer_amd.distributed import ROOT_SHARES, default_shares

    assert default_shares(1) == (1, 1)
    for w in range(2, 9):
        assert default_shares(w) == ROOT_SHARES[w]
        assert default_shares(w, rows=True) == (1, 1)
        assert default_shares(w, dst=1) == (1, 1)
        n_parts, runs = tiling.runs(w, *default_shares(w))
        assert runs[0][0] == 0 and sum(k for _, k in runs) == n_parts


def test_row_tiled_cpu_baseline_runs():
    """oracle/row_tiled.py (bench.py's all-cores CPU baseline): whole frames through
    render_frame_distributed, and the tile-sample mode of the big configs."""
    from oracle import row_tiled

    spec = scenes.readme_spec(48, 27)
    full = row_tiled.time_row_tiled(spec, 3, 2, frames=2)
    assert len(full["times"]) == 2 and full["pixels"] == [48 * 27] * 2
    part = row_tiled.time_row_tiled(spec, 3, 2, frames=2, sub=2, row_block=4)
    assert sum(part["pixels"]) == 48 * 27  # two steps cover the two halves of a 4-way split


def test_cpu_baseline_leg_is_bounded(monkeypatch):
    """bench.py's all-cores CPU leg runs in a child process group with a hard time limit: with a
    worker stuck before its first frame, the leg returns the 1-core baseline plus
    ``all_cores_error`` within the limit instead of hanging the bench line; without it, the
    bounded run returns the row-tiled timing."""
    import time

    import bench

    spec = scenes.readme_spec(48, 27)
    single = {"value": 1.5, "unit": "Mpixels/s", "cores": 1, "kind": "port", "sample": "1-core"}
    ok = bench.cpu_baseline_or_error(spec, 3, 2, 1.0, single, timeout_s=240)
    assert "all_cores_error" not in ok and ok["cores"] == 2 and ok["single_core"] == single
    monkeypatch.setenv("ROW_TILED_STALL_RANK", "1")
    t0 = time.perf_counter()
    out = bench.cpu_baseline_or_error(spec, 3, 2, 1.0, single, timeout_s=30)
    assert time.perf_counter() - t0 < 90
    assert out["value"] == 1.5 and "TimeoutError" in out["all_cores_error"], out
