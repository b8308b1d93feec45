"""The PyTorch custom-op surface ``torch.ops.rt.*``, built in-tree as
``librt_ops.so`` from ``csrc/rt_ops.cpp`` over the C ABI of ``librtx_hip.so``.

    import python_ray_tracer_amd.ops  # registers torch.ops.rt
    ws = torch.zeros(torch.ops.rt.workspace_bytes(n, B), dtype=torch.uint8, device="cuda")
    rgb = torch.ops.rt.render_tile(blob, S, W, H, 1, 1, 0, B, 0, ws)      # [3, W*H] float32

Ops (each raises RuntimeError on a host tensor, a wrong dtype, a non-contiguous tensor or a short
workspace, like a TORCH_CHECK; each runs under a device guard of its input's device, enqueues on
that device's current HIP stream and returns a new tensor):

* ``rt::render_tile(scene, n_spheres, width, height, row_block, n_parts, part, max_bounces,
  out_kind, workspace, stats=None, check=True, part_run=1)`` — get_ray_directions + raytrace_scene
  fused (base.py:91-141) for one interleaved row tile, or the run of ``part_run`` parts from
  ``part`` (a rank's weighted share, distributed.ROOT_SHARES); out_kind 0 = float32 [3, n],
  1 = float64 [3, n], 2 = uint8 [rows, W, 3].
* ``rt::render_frames(scenes, n_spheres, width, height, max_bounces, out_kind, workspace,
  stats=None, check=True)`` — F whole frames in one launch (``scenes``: [F, L], one packed blob per
  row); [F, 3, W*H] colour or [F, H, W, 3] uint8 (HipRenderer.render_batch).
* ``rt::trace(scene, n_spheres, origins, dirs, max_bounces, out_kind, workspace, stats=None,
  check=True)`` — raytrace_scene on arbitrary rays (base.py:91-121); origins [3] (shared) or [3, n].
* ``rt::shade_hits(scene, n_spheres, shape, origins, dirs, t, max_bounces, out_kind, workspace,
  stats=None, check=True)`` — NumpyShader.create for rays hitting sphere ``shape`` at distances
  ``t`` [n] (shader.py:63-112; HipShader.create).
* ``rt::intersect(sphere, origins, dirs)`` — NumpySphere.intersect (shape.py:28-51).
* ``rt::quantize_u8(color)`` — save_image's quantisation (base.py:143-151) -> [n, 3] uint8.
* ``rt::assemble_rows(tiles, width, height, row_block, out_kind, root_run=1, run=1)`` — the
  multi-GPU row un-permute of ``tiles`` [ranks, part_len]: rank 0's run of ``root_run`` parts, each
  other rank's run of ``run`` (tiling.runs; 1, 1 = one part per rank).
* ``rt::status(workspace)`` — reads and clears the sticky RTX_ST_* flags (1 stack overflow,
  2 deferred-list overflow, 4 bad scene); synchronises.
* ``rt::workspace_bytes(n_rays, max_bounces)``.

Error channel of the render ops: with ``check=True`` (the default) a scene blob whose header
disagrees with ``n_spheres`` raises before the launch (one small synchronous header copy), and a
launch that may defer chains past the fast kernel's levels (max_bounces -1 or > 6) reads and clears
the status word afterwards (a synchronisation), raising "maximum recursion depth exceeded" where
HipRenderer raises RecursionError. ``check=False`` keeps the op asynchronous (no host
synchronisation); call ``rt::status(workspace)`` later. ``stats`` and ``workspace`` are declared
as mutated (``Tensor(a!)``, ``Tensor(b!)?``) and every op has a Meta (fake) kernel, so the ops
trace under FakeTensor / torch.compile.

max_bounces -1 is the reference's unbounded recursion. There is no CPU implementation: importing
this module without the built library raises ImportError.
"""

from __future__ import annotations

from pathlib import Path

import torch

from python_ray_tracer_amd.infrastructure.hip import _lib

OPS_LIB = Path(__file__).resolve().parent / "librt_ops.so"
RTX_LIB = Path(__file__).resolve().parent / "librtx_hip.so"  # what librt_ops.so links by $ORIGIN
OPS = ("render_tile", "render_frames", "trace", "shade_hits", "intersect", "quantize_u8", "assemble_rows",
       "status", "workspace_bytes",
       # the row-tiled multi-GPU frame (rtx_tiles_*: render, RCCL gather, assembly in one native call)
       "comm_unique_id", "comm_init", "comm_destroy", "tiles_create", "tiles_submit", "tiles_finish",
       "tiles_destroy")


def load() -> None:
    """Register torch.ops.rt (idempotent)."""
    if hasattr(torch.ops, "rt") and hasattr(torch.ops.rt, "workspace_bytes"):
        try:
            torch.ops.rt.workspace_bytes  # noqa: B018 - resolves only once the library is loaded
            return
        except (AttributeError, RuntimeError):
            pass
    # librt_ops.so resolves the C ABI from the librtx_hip.so beside it ($ORIGIN). A variant library
    # named by RTX_HIP_LIB (tools/ab.py builds) would give the ops and HipRenderer two different
    # kernels in one process: refuse to register rather than mix them.
    if _lib.LIB_PATH.resolve() != RTX_LIB.resolve():
        raise ImportError(f"torch.ops.rt links {RTX_LIB}, but RTX_HIP_LIB selects {_lib.LIB_PATH}: the ops and "
                          "HipRenderer would run different libraries; unset RTX_HIP_LIB to use the ops")
    _lib.load()  # the C ABI first: same file, same handle
    if not OPS_LIB.exists():
        raise ImportError(f"{OPS_LIB} not found; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    torch.ops.load_library(str(OPS_LIB))


load()
