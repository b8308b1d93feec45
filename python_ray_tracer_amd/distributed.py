"""The multi-GPU frame: interleaved row tiles, one gather to the root, one
device un-permute.

The reference renders a frame in one process (``render_image_pipeline``, application.py:43-52);
the north star row-tiles it across the GPUs of a node. Every rank renders its interleaved row
tile (``tiling.py``) straight into a pre-allocated gather buffer (``render_tile(into=...)``); one
``torch.distributed.gather`` moves the tiles to the root (RCCL over xGMI under the "nccl" backend:
the root receives from every peer over its own point-to-point link at once, where a ring
all-gather would be bound by one link); the root un-permutes the rows with one device kernel
(``rtx_assemble_rows``), giving the frame a single-GPU render gives, bit for bit.

``TileGather`` keeps its buffers across frames and lets frames overlap: ``submit(scene, slot)``
enqueues the render and starts the gather asynchronously (the collective runs on the backend's own
stream, after the render), ``finish(slot)`` makes the current stream wait for it and assembles.
With two slots the gather of frame k runs while frame k+1 renders (``bench.py --mode tiles``).
Under gloo (CPU tests, ranks sharing one GPU) tiles travel through host memory and every call is
synchronous.
"""

from __future__ import annotations

import inspect

import numpy as np
import torch

from python_ray_tracer_amd import tiling


class TileGather:
    def __init__(self, renderer, width: int, height: int, *, group=None, row_block: int = 8, dst: int = 0,
                 out: str | None = None, slots: int = 2) -> None:
        import torch.distributed as dist

        self._dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst = int(dst)
        self.gloo = dist.get_backend(group) == "gloo"
        self.r = renderer
        self._into = "into" in inspect.signature(renderer.render_tile).parameters
        self.W, self.H, self.rb = int(width), int(height), int(row_block)
        self.out = "u8" if out == "u8" else None
        dtype = torch.uint8 if self.out == "u8" else getattr(renderer, "color_dtype", torch.float64)
        self.device = torch.device(getattr(renderer, "device", "cpu"))
        self.shape = tiling.tile_shape(self.H, self.W, self.rb, self.world, self.rank, self.out)
        self.n = int(np.prod(self.shape))
        plen = tiling.part_len(self.H, self.W, self.rb, self.world, torch.empty((), dtype=dtype).element_size(),
                               self.out)
        # zero-filled once: the padding beyond a short part's tile is sent but never read
        self.send = [torch.zeros(plen, dtype=dtype, device=self.device) for _ in range(slots)]
        coll = torch.device("cpu") if self.gloo else self.device
        self.recv = ([torch.zeros((self.world, plen), dtype=dtype, device=coll) for _ in range(slots)]
                     if self.rank == self.dst else None)
        # the gather's per-rank views of each receive buffer, built once (not per frame)
        self._recv_lists = [list(b.unbind(0)) for b in self.recv] if self.recv is not None else None
        self._views = [b[:self.n].view(self.shape) for b in self.send]
        self._pending: dict = {}

    def submit(self, scene, slot: int = 0) -> None:
        """Render this rank's tile of ``scene`` into slot ``slot`` and start its gather."""
        if slot in self._pending:
            raise RuntimeError(f"slot {slot} still has a frame in flight: finish() it first")
        buf = self.send[slot]
        view = self._views[slot]
        if self._into:
            self.r.render_tile(scene, self.rb, self.world, self.rank, self.out, into=view)
        else:  # a renderer without into= (test stand-ins): copy its tile in
            view.copy_(self.r.render_tile(scene, self.rb, self.world, self.rank, self.out))
        send = buf.cpu() if (self.gloo and buf.is_cuda) else buf
        gl = self._recv_lists[slot] if self.rank == self.dst else None
        work = self._dist.gather(send, gl, dst=self.dst, group=self.group, async_op=True)
        self._pending[slot] = (work, send)

    def finish(self, slot: int = 0):
        """Wait for slot ``slot``'s gather (a stream wait under nccl) and, on the root, assemble the
        frame: [3, H*W] colour or [H, W, 3] uint8. Other ranks return None."""
        work, _ = self._pending.pop(slot)
        work.wait()
        if self.rank != self.dst:
            return None
        tiles = self.recv[slot]
        if hasattr(self.r, "assemble_rows"):  # HipRenderer: the device un-permute
            return self.r.assemble_rows(tiles, self.W, self.H, self.rb, self.out)
        return tiling.assemble(tiles, self.H, self.W, self.rb, self.out)

    def render(self, scene):
        """One frame, synchronous in program order: submit + finish on slot 0."""
        self.submit(scene, 0)
        return self.finish(0)


# TileGathers cached per renderer (one per frame size / tiling / group / output). Each holds a send
# buffer and, on the root, world x part_len receive buffers (C4 on 8 ranks: ~100 MB of uint8 tiles
# on the root), so the cache is small and evicts the least recently used entry.
TILE_GATHER_CACHE = 4


def tile_gather_for(renderer, scene, *, group=None, row_block: int = 8, dst: int = 0, out=None) -> TileGather:
    """The renderer's cached TileGather for this frame size, tiling and group (buffers persist
    across calls, so a frame sequence allocates nothing per frame). One slot: the synchronous
    render_frame_distributed path never has two frames in flight (bench.py's pipelined tiles mode
    builds its own two-slot TileGather)."""
    import torch.distributed as dist

    W, H = int(scene.camera.width), int(scene.camera.height)
    key = (W, H, int(row_block), int(dst), "u8" if out == "u8" else None, id(group), dist.get_world_size(group),
           getattr(renderer, "color_dtype", None))
    cache = getattr(renderer, "_tile_gathers", None)
    if cache is None:
        cache = {}
        try:
            renderer._tile_gathers = cache
        except AttributeError:  # pragma: no cover - renderer without a __dict__
            pass
    tg = cache.pop(key, None)
    if tg is None:
        while len(cache) >= TILE_GATHER_CACHE:
            cache.pop(next(iter(cache)))  # least recently used (dicts keep insertion order)
        tg = TileGather(renderer, W, H, group=group, row_block=row_block, dst=dst, out=out, slots=1)
    cache[key] = tg  # most recently used last
    return tg
