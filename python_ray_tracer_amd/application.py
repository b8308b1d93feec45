"""Application layer: the plugin surface the HIP backend drops in behind.

Mirrors ``/root/reference/ray_tracer/application.py``:

* ``Renderer`` ABC — ``application.py:7-32`` (``raytrace_scene``, ``get_ray_directions``,
  ``save_image``).
* ``Shader`` ABC — ``application.py:35-40``.
* ``render_image_pipeline(scene, output_path, render_service)`` — ``application.py:43-52``; with one
  process it is the reference's three calls verbatim. When ``torch.distributed`` is initialised
  with more than one rank and the renderer can render row tiles (``HipRenderer.render_tile``), it
  takes the multi-GPU path the north star adds: every rank renders its interleaved row tile
  (``tiling.py``), the tiles are gathered to rank 0 with one collective (RCCL over xGMI on MI355X;
  gloo in the CPU tests), rank 0 un-permutes the rows on the device and writes the PNG.
* ``render_frames`` — the animation driver: frames are sharded round-robin
  over ranks, each rank renders and writes its own frames, no collective.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from pathlib import Path

from python_ray_tracer_amd.domain import Camera, RGBColor, Scene3D, Vector3D


class Renderer(ABC):
    """Calculates the ray directions, traces the rays and saves the result (application.py:7-32)."""

    @abstractmethod
    def raytrace_scene(self, ray_origin: Vector3D, normalized_ray_direction: Vector3D, scene: Scene3D) -> RGBColor:
        pass

    @abstractmethod
    def get_ray_directions(self, camera: Camera):
        pass

    @abstractmethod
    def save_image(self, color: RGBColor, camera: Camera, output_path: Path) -> None:
        pass


class Shader(ABC):
    """Shading calculations (application.py:35-40)."""

    @abstractmethod
    def create(self) -> Vector3D:
        pass


def _dist_world(group):
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    if not (dist.is_available() and dist.is_initialized()):
        return None
    if dist.get_world_size(group) <= 1:
        return None
    return dist


def render_image_pipeline(scene: Scene3D, output_path: Path, render_service: Renderer, *, group=None,
                          row_block: int = 8, gather: str = "color") -> None:
    """application.py:43-52, plus the row-tile / gather path when running on several ranks."""
    dist = _dist_world(group)
    if dist is None or not hasattr(render_service, "render_tile"):
        normalized_ray_destinations = render_service.get_ray_directions(scene.camera)
        color = render_service.raytrace_scene(scene.camera.position, normalized_ray_destinations, scene)
        render_service.save_image(color, scene.camera, output_path)
        return
    frame = render_frame_distributed(scene, render_service, group=group, row_block=row_block, gather=gather)
    if frame is not None:
        if gather == "u8":
            from python_ray_tracer_amd.infrastructure.hip.base import _write_png

            _write_png(frame.cpu().numpy(), output_path)
        else:
            render_service.save_image(_color_of(frame), scene.camera, output_path)


def _color_of(t):
    from python_ray_tracer_amd.infrastructure.hip.base import HipRGBColor

    return HipRGBColor.from_tensor(t)


def render_frame_distributed(scene: Scene3D, render_service, *, group=None, row_block: int = 8, dst: int = 0,
                             gather: str = "color"):
    """Every rank renders its interleaved row tile; one gather to ``dst``; ``dst`` returns the
    frame ([3, H*W] colour, or [H, W, 3] uint8 with ``gather="u8"``), the other ranks None.

    ``render_service.render_tile(scene, row_block, n_parts, part, out[, into])`` renders one tile
    (``HipRenderer.render_tile``). The buffers, the gather and the device un-permute live in
    ``distributed.TileGather`` (cached per renderer and frame shape)."""
    from python_ray_tracer_amd.distributed import tile_gather_for

    out = "u8" if gather == "u8" else None
    return tile_gather_for(render_service, scene, group=group, row_block=row_block, dst=dst, out=out).render(scene)


def render_frames(frames, render_service, output_dir=None, *, group=None, name: str = "frame_{:04d}.png",
                  batch: int = 16):
    """Animation driver: ``frames`` is a sequence of Scene3D (one per frame). Frame k is rendered
    by rank k % world (no collective). Returns {k: colour} for this rank's frames; writes PNGs
    when ``output_dir`` is given (skipping frames whose PNG already exists: resumable).

    With a renderer that has ``render_batch`` (HipRenderer), up to ``batch`` consecutive frames of
    one camera size and sphere count go to the GPU in one launch (rtx_render_frames)."""
    dist = _dist_world(group)
    world = dist.get_world_size(group) if dist else 1
    rank = dist.get_rank(group) if dist else 0
    todo = []
    for k, scene in enumerate(frames):
        if k % world != rank:
            continue
        path = None if output_dir is None else Path(output_dir) / name.format(k)
        if path is not None and path.exists():
            continue
        todo.append((k, scene, path))
    out = {}
    batched = hasattr(render_service, "render_batch") and batch > 1
    i = 0
    while i < len(todo):
        if batched:
            shape = _frame_shape(todo[i][1])
            j = i + 1
            while j < len(todo) and j - i < batch and _frame_shape(todo[j][1]) == shape:
                j += 1
            colors = render_service.render_batch([sc for _, sc, _ in todo[i:j]])
            chunk = [(k, sc, path, _color_of(colors[f])) for f, (k, sc, path) in enumerate(todo[i:j])]
        else:
            k, scene, path = todo[i]
            j = i + 1
            if hasattr(render_service, "render"):
                color = render_service.render(scene)
            else:
                dirs = render_service.get_ray_directions(scene.camera)
                color = render_service.raytrace_scene(scene.camera.position, dirs, scene)
            chunk = [(k, scene, path, color)]
        for k, scene, path, color in chunk:
            if path is not None:
                render_service.save_image(color, scene.camera, path)
            out[k] = color
        i = j
    return out


def _frame_shape(scene):
    return int(scene.camera.width), int(scene.camera.height), len(list(scene.shapes))
