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

Under RCCL with ``HipRenderer`` (``native``, the default there) a frame is ONE native call per rank
(``rtx_tiles_submit``, csrc/rtx_tiles.hip): the render, the peers' RCCL sends / the root's receives
(the library's own communicator over the same librccl torch loaded) and the root's assembly are
enqueued without Python between them, on the caller's stream and the plan's collective stream.
"""

from __future__ import annotations

import inspect

import numpy as np
import torch

from python_ray_tracer_amd import tiling


# Block slots a gathering plan's persistent renders leave free for the previous frame's RCCL kernels
# (RTX_F_RESERVE). One GPU, C4 through a loopback plan (the tile sent to itself over RCCL, 100 MB,
# then assembled) beside the next frame's render: 2,256-2,273 us per step with no reserve, 2,188-2,207
# with 64 (16: 2,389; 128: 2,309; 256: 2,569), against 2,060 without the gather
# (profiles/r4d_gather_ab, r4e_gather_ab); capping RCCL's CTAs at 2, 4 or 8 changed nothing.
COMM_RESERVE_BLOCKS = 64


# Shares (root_run, run) of the row-tiled frame by world size: the root also receives every part and
# assembles the frame beside its next render (~0.33 us of render time per MB of that HBM traffic,
# DESIGN.md §6), so it renders fewer rows than a peer. Chosen on the C4 part emulation (one GPU,
# profiles/r4_shares_C4.json: slowest of root render + its traffic and a peer's render): 2 ranks
# 8:9 (1,086 us against 1,145 equal), 4 ranks 3:4 (558 against 639), 8 ranks 1:2 (296 against 396);
# 3, 5, 6 and 7 ranks interpolated, not measured.
ROOT_SHARES = {2: (8, 9), 3: (3, 4), 4: (3, 4), 5: (2, 3), 6: (2, 3), 7: (1, 2), 8: (1, 2)}


def default_shares(world: int, dst: int = 0, rows: bool = False) -> tuple:
    """(root_run, run) a TileGather takes unless told otherwise: ROOT_SHARES with the root at rank 0;
    even shares for a root elsewhere, and for RTX_TILES_ROWS (each row block of a part travels on
    its own into the frame; the native plan takes runs of one part only)."""
    if rows or dst != 0:
        return (1, 1)
    return ROOT_SHARES.get(int(world), (1, 1))


# RCCL communicators of the native path, one per (process group, rank, device): creating one costs
# a rendezvous, so TileGathers of the same group share it for the life of the process
_COMMS: dict = {}


def rccl_comm(group, root: int, device, max_ctas: int | None = None):
    """The library's RCCL communicator over ``group`` (rtx_comm_init): the root's ncclUniqueId is
    broadcast over the group itself. Collective: every rank of the group calls it. ``max_ctas``
    (default: env RTX_COMM_MAX_CTAS, else RCCL's own choice) caps the blocks of its kernels."""
    import os

    import ctypes

    import torch.distributed as dist

    from python_ray_tracer_amd.infrastructure.hip import _lib as L

    pg = group if group is not None else dist.group.WORLD
    world, rank = dist.get_world_size(pg), dist.get_rank(pg)
    if max_ctas is None:
        max_ctas = int(os.environ.get("RTX_COMM_MAX_CTAS", "0"))
    key = (getattr(pg, "group_name", id(pg)), world, rank, torch.device(device).index, int(max_ctas))
    comm = _COMMS.get(key)
    if comm is not None:
        return comm
    lib = L.load()
    L.rccl_load()
    uid = (ctypes.c_char * L.UNIQUE_ID_BYTES)()
    if rank == root:
        L.check(lib.rtx_comm_unique_id(uid), "rtx_comm_unique_id")
    obj = [bytes(uid) if rank == root else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(pg, root), group=pg, device=torch.device(device))
    uid = (ctypes.c_char * L.UNIQUE_ID_BYTES).from_buffer_copy(obj[0])
    c = ctypes.c_void_p()
    with torch.cuda.device(device):
        L.check(lib.rtx_comm_init(uid, world, rank, int(max_ctas), ctypes.byref(c)), "rtx_comm_init")
    _COMMS[key] = c.value
    return c.value


class TileGather:
    def __init__(self, renderer, width: int, height: int, *, group=None, row_block: int = 8, dst: int = 0,
                 out: str | None = None, slots: int = 2, native: bool | None = None,
                 persistent_frames: bool = False, loopback: bool = False, comm_reserve: int | None = None,
                 rows: bool | None = None, shares: tuple | None = None, timed: bool = False) -> None:
        """``native``: drive each frame through rtx_tiles_submit (default: under RCCL with a
        renderer that has ``submit_tiles``); False keeps torch.distributed.gather. ``persistent_frames``
        (native root): assemble every frame of a slot into one buffer kept by the slot, so a frame
        returned by finish(slot) is overwritten by that slot's next frame (the bench); otherwise each
        frame gets a new tensor. ``loopback`` (native, one rank): the tile still travels through RCCL
        (sent to and received from the rank itself), the gather path on one GPU (tests).
        ``comm_reserve``: block slots every persistent render of a gathering plan leaves free for the
        previous frame's RCCL kernels (RTX_F_RESERVE; default COMM_RESERVE_BLOCKS). ``rows`` (native,
        uint8 frames): every row block travels on its own straight into the root's frame
        (RTX_TILES_ROWS), with no assembly pass on the root. Off by default: RCCL charges ~2.7 us per
        operation (one GPU, C4 loopback: 5,480 us per step with row blocks of 8 rows, 2,837 with 32,
        against 2,190 gathered whole and assembled). ``shares`` = (root_run, run): rank 0 renders
        root_run parts and every other rank run parts of a root_run + (world - 1) run interleave
        (tiling.runs); default ``default_shares``: ROOT_SHARES by world size (the root also receives
        and assembles every frame, so it takes a smaller share; the root must then be rank 0), even
        shares with ``rows`` (which moves parts of one run each). ``timed`` (native plans that
        gather): timing events around every gather (RTX_TILES_TIMED), read by ``timing(slot)``."""
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
        if shares is None:
            shares = default_shares(self.world, self.dst, bool(rows) and self.out == "u8")
        self.root_run, self.run = int(shares[0]), int(shares[1])
        if self.root_run != self.run and self.dst != 0:
            raise ValueError("unequal shares need the root at rank 0")
        if rows and self.out == "u8" and (self.root_run, self.run) != (1, 1):
            raise ValueError("rows=True (RTX_TILES_ROWS) moves parts of one run each: shares must be (1, 1)")
        self.n_parts, runs = tiling.runs(self.world, self.root_run, self.run)
        self.first, self.my_run = runs[self.rank]
        self.shape = tiling.tile_shape(self.H, self.W, self.rb, self.n_parts, self.first, self.out, self.my_run)
        self.n = int(np.prod(self.shape))
        plen = tiling.part_len(self.H, self.W, self.rb, self.world, torch.empty((), dtype=dtype).element_size(),
                               self.out, self.root_run, self.run)
        self._pending: dict = {}
        self.plan = None
        if native is None:
            native = not self.gloo and hasattr(renderer, "submit_tiles")
        if native:
            self._init_native(dtype, plen, slots, persistent_frames, loopback and self.world == 1,
                              COMM_RESERVE_BLOCKS if comm_reserve is None else int(comm_reserve),
                              bool(rows) and self.out == "u8", bool(timed))
            return
        # zero-filled once: the padding beyond a short part's tile is sent but never read
        self.send = [torch.zeros(plen, dtype=dtype, device=self.device) for _ in range(slots)]
        coll = torch.device("cpu") if self.gloo else self.device
        self.recv = ([torch.zeros((self.world, plen), dtype=dtype, device=coll) for _ in range(slots)]
                     if self.rank == self.dst else None)
        # the gather's per-rank views of each receive buffer, built once (not per frame)
        self._recv_lists = [list(b.unbind(0)) for b in self.recv] if self.recv is not None else None
        self._views = [b[:self.n].view(self.shape) for b in self.send]

    def _init_native(self, dtype, plen, slots, persistent_frames, loop, reserve, rows, timed=False) -> None:
        import ctypes

        from python_ray_tracer_amd.infrastructure.hip import _lib as L

        if not 1 <= slots <= L.TILES_MAX_SLOTS:
            raise ValueError(f"slots must be 1..{L.TILES_MAX_SLOTS}")
        self._L = L
        self._lib = L.load()
        root = self.rank == self.dst
        self.send = ([torch.zeros(plen, dtype=dtype, device=self.device) for _ in range(slots)]
                     if not root or loop else [])
        gathers = self.world > 1 or loop
        self.rows = rows and gathers
        self.timed = timed and gathers
        self.part_bytes = plen * torch.empty((), dtype=dtype).element_size()
        # RTX_TILES_ROWS: the root keeps only its own tile (the peers' blocks land in the frame)
        self.recv = ([torch.zeros((1 if self.rows else self.world, plen), dtype=dtype, device=self.device)
                      for _ in range(slots)] if root and gathers else None)
        self.frame_shape = (self.H, self.W, 3) if self.out == "u8" else (3, self.H * self.W)
        self._dtype = dtype
        self.frames = ([torch.empty(self.frame_shape, dtype=dtype, device=self.device) for _ in range(slots)]
                       if root and persistent_frames else None)
        comm = rccl_comm(self.group, self.dst, self.device) if self.world > 1 or loop else None
        ptrs = ctypes.c_void_p * slots
        send = ptrs(*[b.data_ptr() for b in self.send]) if self.send else None
        recv = ptrs(*[b.data_ptr() for b in self.recv]) if self.recv else None
        kind = L.OUT_U8_HWC if self.out == "u8" else (L.OUT_F64_SOA if dtype == torch.float64 else L.OUT_F32_SOA)
        plan = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check(self._lib.rtx_tiles_create(comm, self.world, self.rank, self.dst, self.W, self.H, self.rb, kind,
                                               slots, send, recv, plen * torch.empty((), dtype=dtype).element_size(),
                                               self.root_run, self.run,
                                               (L.TILES_LOOPBACK if loop else 0) | (L.TILES_ROWS if self.rows else 0)
                                               | (L.TILES_TIMED if self.timed else 0)
                                               | ((reserve & 0xFFF) << L.F_RESERVE_SHIFT),
                                               ctypes.byref(plan)),
                    "rtx_tiles_create")
        self.plan = plan.value

    def __del__(self):
        plan, self.plan = getattr(self, "plan", None), None
        if plan is not None:
            try:
                self._lib.rtx_tiles_destroy(plan)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass

    def submit(self, scene, slot: int = 0) -> None:
        """Render this rank's tile of ``scene`` into slot ``slot`` and start its gather."""
        if slot in self._pending:
            raise RuntimeError(f"slot {slot} still has a frame in flight: finish() it first")
        if self.plan is not None:
            if (self.world > 1 or self.send) and torch.cuda.is_current_stream_capturing():
                # RCCL traffic inside a HIP graph capture: hipStreamEndCapture overflows the stack in
                # torch's bundled HIP runtime (unbounded recursion over its per-stream capture lists;
                # the trigger is the RCCL group, not the plan's fork/join: DESIGN.md §6, round 6), so a
                # gathering plan is refused up front; a one-rank plan (no RCCL operation) captures and
                # replays
                raise RuntimeError("a gathering TileGather plan cannot be captured into a HIP graph "
                                   "(RCCL send/recv under stream capture); run it eagerly")
            frame = None
            if self.rank == self.dst:
                frame = (self.frames[slot] if self.frames is not None
                         else torch.empty(self.frame_shape, dtype=self._dtype, device=self.device))
            self.r.submit_tiles(self.plan, slot, scene, self.rb, self.n_parts, self.first, frame, part_run=self.my_run)
            self._pending[slot] = (None, frame)
            return
        buf = self.send[slot]
        view = self._views[slot]
        if self._into:
            self.r.render_tile(scene, self.rb, self.n_parts, self.first, self.out, into=view, part_run=self.my_run)
        else:  # a renderer without into= (test stand-ins): copy its tile in
            kw = {"part_run": self.my_run} if self.my_run != 1 else {}
            view.copy_(self.r.render_tile(scene, self.rb, self.n_parts, self.first, self.out, **kw))
        send = buf.cpu() if (self.gloo and buf.is_cuda) else buf
        gl = self._recv_lists[slot] if self.rank == self.dst else None
        work = self._dist.gather(send, gl, dst=self.dst, group=self.group, async_op=True)
        self._pending[slot] = (work, send)

    def finish(self, slot: int = 0):
        """Wait for slot ``slot``'s gather (a stream wait under nccl) and, on the root, assemble the
        frame: [3, H*W] colour or [H, W, 3] uint8. Other ranks return None."""
        work, frame = self._pending.pop(slot)
        if self.plan is not None:
            with torch.cuda.device(self.device):
                self._L.check(self._lib.rtx_tiles_finish(self.plan, slot,
                                                         self._L.stream_handle(torch.cuda.current_stream(self.device))),
                              "rtx_tiles_finish")
            return frame
        work.wait()
        if self.rank != self.dst:
            return None
        tiles = self.recv[slot]
        if hasattr(self.r, "assemble_rows"):  # HipRenderer: the device un-permute
            return self.r.assemble_rows(tiles, self.W, self.H, self.rb, self.out, self.root_run, self.run)
        return tiling.assemble(tiles, self.H, self.W, self.rb, self.out, self.root_run, self.run)

    def timing(self, slot: int = 0) -> dict:
        """The measured gather of slot ``slot``'s latest frame on this rank (a ``timed`` native plan
        that gathers; rtx_tiles_timing, synchronising): ``gather_ms`` from this rank's tile rendered
        to its RCCL group complete (a peer: its part delivered to the root; the root: every peer's
        part received), ``assemble_ms`` the root's assembly, ``bytes`` this rank's RCCL traffic per
        frame (a peer sends part_bytes; the root receives (world - 1) part_bytes)."""
        import ctypes

        if self.plan is None or not getattr(self, "timed", False):
            raise RuntimeError("timing() needs a native plan that gathers, created with timed=True")
        g, a = ctypes.c_float(), ctypes.c_float()
        with torch.cuda.device(self.device):
            self._L.check(self._lib.rtx_tiles_timing(self.plan, int(slot), ctypes.byref(g), ctypes.byref(a)),
                          "rtx_tiles_timing")
        peers = max(self.world - 1, 1)
        nbytes = self.part_bytes * (peers if self.rank == self.dst else 1)
        return {"gather_ms": float(g.value), "assemble_ms": float(a.value), "bytes": int(nbytes),
                "part_bytes": int(self.part_bytes)}

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
