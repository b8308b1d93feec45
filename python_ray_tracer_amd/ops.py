"""The PyTorch custom-op surface ``torch.ops.rt.*``, built in-tree as
``librt_ops.so`` from ``csrc/rt_ops.cpp`` over the C ABI of ``librtx_hip.so``.

    import python_ray_tracer_amd.ops  # registers torch.ops.rt
    ws = torch.zeros(torch.ops.rt.workspace_bytes(n, B), dtype=torch.uint8, device="cuda")
    rgb = torch.ops.rt.render_tile(blob, S, W, H, 1, 1, 0, B, 0, ws)      # [3, W*H] float32

Ops (each raises RuntimeError on a host tensor, a wrong dtype, a non-contiguous tensor or a short
workspace, like a TORCH_CHECK; each enqueues on the current HIP stream and returns a new tensor):

* ``rt::render_tile(scene, n_spheres, width, height, row_block, n_parts, part, max_bounces,
  out_kind, workspace, stats=None)`` — get_ray_directions + raytrace_scene fused
  (base.py:91-141) for one interleaved row tile; out_kind 0 = float32 [3, n], 1 = float64 [3, n],
  2 = uint8 [rows, W, 3].
* ``rt::trace(scene, n_spheres, origins, dirs, max_bounces, out_kind, workspace, stats=None)`` —
  raytrace_scene on arbitrary rays (base.py:91-121); origins [3] (shared) or [3, n].
* ``rt::intersect(sphere, origins, dirs)`` — NumpySphere.intersect (shape.py:28-51).
* ``rt::quantize_u8(color)`` — save_image's quantisation (base.py:143-151) -> [n, 3] uint8.
* ``rt::assemble_rows(tiles, width, height, row_block, out_kind)`` — the multi-GPU row un-permute.
* ``rt::workspace_bytes(n_rays, max_bounces)``.

max_bounces -1 is the reference's unbounded recursion. There is no CPU implementation: importing
this module without the built library raises ImportError.
"""

from __future__ import annotations

from pathlib import Path

import torch

from python_ray_tracer_amd.infrastructure.hip import _lib

OPS_LIB = Path(__file__).resolve().parent / "librt_ops.so"
OPS = ("render_tile", "trace", "intersect", "quantize_u8", "assemble_rows", "workspace_bytes")


def load() -> None:
    """Register torch.ops.rt (idempotent)."""
    if hasattr(torch.ops, "rt") and hasattr(torch.ops.rt, "workspace_bytes"):
        try:
            torch.ops.rt.workspace_bytes  # noqa: B018 - resolves only once the library is loaded
            return
        except (AttributeError, RuntimeError):
            pass
    _lib.load()  # the C ABI first: same file, same handle (librt_ops.so links it by $ORIGIN)
    if not OPS_LIB.exists():
        raise ImportError(f"{OPS_LIB} not found; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    torch.ops.load_library(str(OPS_LIB))


load()
