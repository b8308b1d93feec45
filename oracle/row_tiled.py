"""CPU ORACLE, all host cores — test / baseline infrastructure only, NOT the product path.

The north star asks for the NumPy CPU path "timed on the GPU box's own host cores"; the reference
itself is single-threaded NumPy. This runs the oracle (``numpy_oracle``, the
reference's algorithm) row-tiled over P processes through the product's own multi-rank frame path
(``application.render_frame_distributed`` over gloo): every process renders its interleaved row
tile with the oracle (one core each), the tiles are gathered to rank 0 and un-permuted there.
Only ``bench.py``'s ``cpu_baseline`` leg and ``tests/`` use it.
"""

from __future__ import annotations

import json
import os
import socket
import tempfile
import time

import numpy as np


class OracleTileRenderer:
    """The ``render_tile`` contract of HipRenderer, computed by the oracle on the CPU (float64)."""

    def __init__(self, max_bounces):
        self.B = max_bounces

    def render_tile(self, scene, row_block, n_parts, part, out=None, part_run=1):
        import torch

        from oracle import numpy_oracle as O
        from python_ray_tracer_amd import tiling

        sc = O.scene_from_objects(scene)
        rows = tiling.tile_rows(sc.height, row_block, n_parts, part, part_run)
        t = O.render_rows(sc, rows, self.B)
        if out == "u8":
            return torch.from_numpy(np.ascontiguousarray(O.to_uint8(t, sc.width, len(rows))))
        return torch.from_numpy(np.ascontiguousarray(t))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, spec, B, frames, outfile, row_block, sub):
    # gloo reports its connections on fd 1: keep the parent's stdout (bench.py's one JSON line) clean
    os.dup2(2, 1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from python_ray_tracer_amd import scenes, tiling
    from python_ray_tracer_amd.application import render_frame_distributed

    import datetime

    # a bound on every gloo rendezvous and collective: a sibling that died cannot hold this one
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))
    try:
        if os.environ.get("ROW_TILED_STALL_RANK") == str(rank):  # test hook: a stuck worker (tests/)
            time.sleep(3600)
        scene = scenes.build_scene(spec)
        r = OracleTileRenderer(B)
        times, pixels = [], []
        W, H = int(spec["camera"]["width"]), int(spec["camera"]["height"])
        for k in range(frames):
            dist.barrier()
            t0 = time.perf_counter()
            if sub == 1:  # the whole frame through the product's multi-rank path
                render_frame_distributed(scene, r, row_block=row_block)
                px = W * H
            else:  # a sample: rank r renders part r * sub + j of a (world * sub)-way split, one gather
                part = rank * sub + k % sub
                tile = r.render_tile(scene, row_block, world * sub, part)
                rmax = tiling.max_local_rows(H, row_block, world * sub)
                buf = torch.zeros((3, rmax * W), dtype=tile.dtype)
                buf[:, :tile.shape[1]] = tile
                dist.gather(buf, [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None, dst=0)
                px = sum(tiling.n_local_rows(H, row_block, world * sub, q * sub + k % sub) for q in range(world)) * W
            dist.barrier()  # every rank's tile done (and gathered): the sample is complete on rank 0
            times.append(time.perf_counter() - t0)
            pixels.append(px)
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump({"times": times, "pixels": pixels}, f)
    finally:
        dist.destroy_process_group()


def time_row_tiled(spec: dict, max_bounces, procs: int, frames: int = 3, row_block: int = 8, sub: int = 1) -> dict:
    """Wall time per frame of the row-tiled oracle on ``procs`` processes (one core each):
    render + gather + un-permute, process start-up and imports excluded. ``sub`` > 1 times a
    sample instead of whole frames: each step, every process renders one part of a
    (procs * sub)-way interleaved split (1/sub of the frame in total). Returns
    {"times": [...], "pixels": [...]} per step."""
    # stdlib multiprocessing (spawn): this process itself never imports torch, so under
    # run_bounded only the workers hold the GPU runtime open (the box allows 16 such processes)
    import multiprocessing as mp

    old = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in old:
        os.environ[k] = "1"  # one core per process (NumPy's elementwise ufuncs are single-threaded anyway)
    try:
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "times.json")
            ctx = mp.get_context("spawn")
            port = _free_port()
            ps = [ctx.Process(target=_worker, args=(r, procs, port, spec, max_bounces, frames, out, row_block, sub))
                  for r in range(procs)]
            for p in ps:
                p.start()
            # poll: when one worker fails, the others would wait in the gloo rendezvous or the
            # gather until gloo's own timeout, so they are terminated at once
            try:
                while any(p.is_alive() for p in ps):
                    if any(p.exitcode not in (None, 0) for p in ps):
                        break
                    time.sleep(0.05)
            finally:
                for p in ps:
                    if p.is_alive():
                        p.terminate()
                for p in ps:
                    p.join()
            bad = [(r, p.exitcode) for r, p in enumerate(ps) if p.exitcode != 0]
            if bad:
                raise RuntimeError(f"row-tiled workers failed (rank, exit code): {bad}")
            with open(out) as f:
                return json.load(f)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_bounded(spec: dict, max_bounces, procs: int, frames: int, sub: int, timeout_s: float,
                row_block: int = 8) -> dict:
    """time_row_tiled in a child process (its own session) with a hard time limit: a worker stuck in
    the gloo rendezvous or the gather cannot hang the caller (bench.py's cpu_baseline leg). On
    timeout the child's whole process group — the child and its spawned workers — is killed and
    TimeoutError raised."""
    import signal
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as d:
        args = os.path.join(d, "args.json")
        out = os.path.join(d, "out.json")
        with open(args, "w") as f:
            json.dump({"spec": spec, "B": max_bounces, "procs": procs, "frames": frames, "sub": sub,
                       "row_block": row_block, "out": out}, f)
        # stdout to stderr: the caller's stdout carries bench.py's one JSON line
        p = subprocess.Popen([sys.executable, "-m", "oracle.row_tiled", args], cwd=repo, stdout=sys.stderr,
                             start_new_session=True)
        try:
            rc = p.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)  # the group this call created (start_new_session)
            p.wait()
            raise TimeoutError(f"row-tiled CPU baseline exceeded {timeout_s:.0f}s; its process group was killed")
        if rc != 0:
            raise RuntimeError(f"row-tiled CPU baseline exited with {rc}")
        with open(out) as f:
            return json.load(f)


def _main(argv) -> None:
    # through the importable module, so the spawned workers unpickle oracle.row_tiled._worker
    from oracle.row_tiled import time_row_tiled

    with open(argv[0]) as f:
        a = json.load(f)
    res = time_row_tiled(a["spec"], a["B"], a["procs"], frames=a["frames"], row_block=a["row_block"], sub=a["sub"])
    with open(a["out"], "w") as f:
        json.dump(res, f)


def host_cores() -> int:
    """CPUs this process may run on (the GPU box shares a large host: its cgroup/affinity share)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover
        return os.cpu_count() or 1


if __name__ == "__main__":
    import sys

    _main(sys.argv[1:])
