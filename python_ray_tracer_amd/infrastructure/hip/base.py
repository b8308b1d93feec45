"""HIP backend: vector containers and ``HipRenderer``, the drop-in for ``NumpyRenderer``.

Reference surface (``/root/reference/ray_tracer/infrastructure/numpy/base.py``):

* ``FARAWAY``                                  — ``base.py:12``
* ``NumpyVector3D`` / ``NumpyVectorArray3D`` / ``NumpyRGBColor`` — ``base.py:28-87``
  -> ``HipVector3D`` / ``HipVectorArray3D`` / ``HipRGBColor``: the same SoA container, whose
  components may be Python scalars, NumPy arrays or device tensors. The algebra (``dot``, ``norm``,
  ``extract``, ``place`` …) keeps the reference semantics for API compatibility; it is convenience,
  not the hot path — the renderer never computes through it.
* ``NumpyRenderer``                            — ``base.py:90-151`` -> ``HipRenderer``:
  ``get_ray_directions`` returns a lazy ``HipCameraRays`` batch; ``raytrace_scene`` on that batch
  launches one fused kernel (ray generation + all bounce levels, ``rtx_render_camera``); on any other
  rays it launches ``rtx_trace_rays``; ``save_image`` quantises on the device
  (``rtx_quantize_u8``) and writes the PNG with Pillow like ``base.py:143-151``.

Differences from the reference, all deliberate and documented in DESIGN.md:
* ``HipRenderer(max_bounces=None)`` (the default) follows the reference's unbounded recursion up to
  ``UNBOUNDED_LEVELS`` (333) levels and raises ``RecursionError`` beyond, where Python's recursion
  limit would stop the reference. ``max_bounces=B`` caps it (levels 0..B shaded, level B+1 black).
* ``color_dtype`` float64 (default, the reference dtype) or float32.
"""

from __future__ import annotations

import ctypes
import numbers
import os
from pathlib import Path

import numpy as np
import torch

from python_ray_tracer_amd.application import Renderer
from python_ray_tracer_amd.domain import Camera, RGBColor, Vector3D
from python_ray_tracer_amd.tiling import n_local_rows

from . import _lib as L
from .scene_pack import camera_words, pack_key, scene_key

FARAWAY = 1.0e39  # base.py:12


def _is_tensor(x) -> bool:
    return isinstance(x, torch.Tensor)


def _sqrt(x):
    # correctly rounded, like np.sqrt: torch's CPU sqrt is not (its SIMD path is off by up to 1 ulp)
    if _is_tensor(x):
        if x.device.type == "cpu":
            return torch.from_numpy(np.sqrt(x.detach().numpy()))
        return torch.sqrt(x)
    return np.sqrt(x)


def _where(c, a, b):
    if _is_tensor(c):
        return torch.where(c, torch.as_tensor(a, dtype=torch.float64, device=c.device),
                           torch.as_tensor(b, dtype=torch.float64, device=c.device) if not _is_tensor(b) else b)
    return np.where(c, a, b)


class HipVector3D(Vector3D):
    """SoA 3-vector (reference ``NumpyVector3D``, base.py:28-79)."""

    def __init__(self, x, y, z) -> None:
        (self.x, self.y, self.z) = (x, y, z)

    def dot(self, other):
        return (self.x * other.x) + (self.y * other.y) + (self.z * other.z)  # base.py:34-35

    def __abs__(self):
        return self.dot(self)  # squared norm, base.py:37-38

    def components(self):
        return (self.x, self.y, self.z)

    def __mul__(self, other):
        if isinstance(other, HipVector3D):
            return HipVector3D(self.x * other.x, self.y * other.y, self.z * other.z)
        return HipVector3D(self.x * other, self.y * other, self.z * other)

    def __add__(self, other):
        return HipVector3D(self.x + other.x, self.y + other.y, self.z + other.z)

    def __sub__(self, other):
        return HipVector3D(self.x - other.x, self.y - other.y, self.z - other.z)

    def __neg__(self):
        return HipVector3D(-self.x, -self.y, -self.z)

    def __truediv__(self, other):
        return HipVector3D(self.x / other, self.y / other, self.z / other)

    def norm(self):
        mag = _sqrt(self.dot(self))  # base.py:61-64
        return self * (1.0 / _where(mag == 0, 1, mag))

    def extract(self, cond):
        if isinstance(cond, numbers.Number):
            return self
        return HipVectorArray3D(*(_extract(cond, c) for c in self.components()))

    def place(self, cond):
        out = []
        for c in self.components():
            if _is_tensor(cond):
                r = torch.zeros(cond.shape, dtype=torch.float64, device=cond.device)
                r[cond] = torch.as_tensor(c, dtype=torch.float64, device=cond.device)
            else:
                r = np.zeros(np.shape(cond))
                np.place(r, cond, c)
            out.append(r)
        return HipVector3D(*out)

    # --- device helpers -------------------------------------------------------------------
    def is_scalar(self) -> bool:
        return all(np.ndim(c) == 0 and not (_is_tensor(c) and c.dim() > 0) for c in self.components())

    def to_tensor(self, device, n: int | None = None) -> torch.Tensor:
        """[3] (shared/scalar) or [3, n] float64 contiguous device tensor."""
        comps = self.components()
        if self.is_scalar():
            vals = [float(c) for c in comps]
            return torch.tensor(vals, dtype=torch.float64).to(device)
        cols = []
        for c in comps:
            t = c if _is_tensor(c) else torch.from_numpy(np.ascontiguousarray(np.asarray(c, dtype=np.float64)))
            t = t.to(device=device, dtype=torch.float64)
            cols.append(t.reshape(-1) if t.dim() else t.expand(n if n is not None else 1))
        length = max(int(c.numel()) for c in cols)
        cols = [c.expand(length) if c.numel() == 1 else c for c in cols]
        return torch.stack(cols).contiguous()

    def numpy(self):
        return tuple(c.detach().cpu().numpy() if _is_tensor(c) else np.asarray(c) for c in self.components())


def _extract(cond, x):
    if isinstance(x, numbers.Number):
        return x
    if _is_tensor(x):
        return x[cond]
    return np.extract(cond, x)


class HipVectorArray3D(HipVector3D):
    """Reference ``NumpyVectorArray3D`` (base.py:82-83)."""


class HipRGBColor(HipVector3D, RGBColor):
    """Reference ``NumpyRGBColor`` (base.py:86-87). ``HipRenderer`` returns one backed by a single
    ``[3, n]`` device tensor (``.data``); ``.x/.y/.z`` are its rows."""

    @classmethod
    def from_tensor(cls, t: torch.Tensor) -> HipRGBColor:
        c = cls(t[0], t[1], t[2])
        c.data = t
        return c


class HipCameraRays(HipVectorArray3D):
    """Lazy result of ``HipRenderer.get_ray_directions`` (base.py:123-141).

    ``raytrace_scene`` on this batch never materialises it: ray generation is fused into the render
    kernel. Reading ``.x/.y/.z`` materialises the float64 ``[3, W*H]`` tensor on the device (the exact
    ``np.linspace`` / ``norm`` arithmetic of the reference)."""

    def __init__(self, renderer: HipRenderer, camera: Camera) -> None:  # noqa: D107
        self._renderer = renderer
        self.camera = camera
        self._data = None

    def _materialise(self) -> torch.Tensor:
        if self._data is None:
            self._data = self._renderer._ray_directions(self.camera)
        return self._data

    @property
    def data(self) -> torch.Tensor:
        return self._materialise()

    x = property(lambda self: self._materialise()[0])
    y = property(lambda self: self._materialise()[1])
    z = property(lambda self: self._materialise()[2])


_OUT_KIND = {torch.float32: L.OUT_F32_SOA, torch.float64: L.OUT_F64_SOA}


def _on_device(method):
    """Run a launching method with the renderer's device current: the library sizes grids by the
    current device's CUs and occupancy and launches there, so a HipRenderer(device="cuda:1") must
    not depend on which device the caller made current."""
    import functools

    @functools.wraps(method)
    def run(self, *args, **kwargs):
        idx = self.device.index
        prev = torch.cuda.current_device()
        if prev == idx:  # the common case: no device switch (and no context manager's cost)
            return method(self, *args, **kwargs)
        torch.cuda.set_device(idx)
        try:
            return method(self, *args, **kwargs)
        finally:
            torch.cuda.set_device(prev)
    return run


class HipRenderer(Renderer):
    """MI355X renderer behind the reference ``Renderer`` plugin surface (application.py:7-32)."""

    def __init__(self, max_bounces: int | None = None, *, color_dtype: torch.dtype = torch.float64,
                 device=None, collect_stats: bool = False, learn_tile_order: bool = True,
                 fast_textures: bool = True) -> None:
        self._lib = L.load()
        if not torch.cuda.is_available():
            raise RuntimeError("HipRenderer needs a ROCm GPU (torch.cuda.is_available() is False); there is no CPU path")
        if max_bounces is not None and (int(max_bounces) != max_bounces or max_bounces < 0):
            raise ValueError(f"max_bounces must be None or a non-negative int, got {max_bounces!r}")
        if color_dtype not in _OUT_KIND:
            raise ValueError(f"color_dtype must be float32 or float64, got {color_dtype}")
        self.max_bounces = None if max_bounces is None else int(max_bounces)
        self.color_dtype = color_dtype
        self.device = _resolve_device(device)
        self._scene_cache: dict = {}
        # camera renders known to defer no ray (or probing): see _general_plan
        self._defers: dict = {}
        # camera launches: the dispatch order learnt per (scene, tile, cap), see _sched_plan
        self.learn_tile_order = bool(learn_tile_order)
        self._sched: dict = {}
        # uncapped camera renders whose status came back clean (see _check_status)
        self._clean: dict = {}
        # scenes with image textures: the fast kernel's texturing build (RTX_F_IMAGES) shades them;
        # False defers those pixels to the general kernel (same colours)
        self.fast_textures = bool(fast_textures)
        self._ws = None
        self._graph_pins: dict = {}  # data_ptr -> tensor a captured launch points at (_tile_launch)
        self.stats_buffer = torch.zeros(L.S_WORDS, dtype=torch.int64, device=self.device) if collect_stats else None

    # ---------------------------------------------------------------- plumbing
    @property
    def _bounces_arg(self) -> int:
        return L.UNBOUNDED if self.max_bounces is None else self.max_bounces

    def _stream(self) -> int:
        return L.stream_handle(torch.cuda.current_stream(self.device))

    def scene_blob(self, scene) -> tuple[torch.Tensor, int]:
        """Packed scene on the device, cached by content: the key is every value the render reads
        from the scene (scene_pack.scene_key), so a mutated scene is re-packed and re-uploaded."""
        return self._scene_entry(scene_key(scene))

    def _scene_entry(self, key) -> tuple[torch.Tensor, int]:
        hit = self._scene_cache.get(key)
        if hit is None:
            blob = pack_key(*key)
            hit = (torch.from_numpy(blob).pin_memory().to(self.device, non_blocking=True), int(blob[L.H_NSPH]))
            if len(self._scene_cache) >= 16:
                self._scene_cache.pop(next(iter(self._scene_cache)))
            self._scene_cache[key] = hit
        return hit

    def workspace(self, n: int) -> torch.Tensor:
        need = int(self._lib.rtx_workspace_bytes(int(n), self._bounces_arg))
        if self._ws is None or self._ws.numel() < need:
            # zero-filled once; every call leaves its counters zeroed again (include/rtx_hip.h)
            self._ws = torch.zeros(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def _general_plan(self, key):
        """(flags, probe) for a camera render identified by ``key`` (scene content, tile, cap).
        The tie/deep kernel (k_render_general) runs after every fast launch (and, uncapped, the
        continuation pass before it); when a frame
        defers no ray it only reads three zero counters, but it is still a launch (about 2.4% of a
        1080p C2 frame). The first render of a key probes: the library writes the launch's
        deferred count into a device word, copied to pinned memory behind an event. Once that
        event has completed, a render of the same key — the same blob content, so the same rays,
        ties and chains: the kernels are deterministic — passes RTX_F_NO_GENERAL if the count was
        0. Nothing here synchronises: until the probe has landed, renders launch the general
        kernel as before."""
        st = self._defers.get(key)
        if st is True:
            return L.F_NO_GENERAL, None
        if st is False or torch.cuda.is_current_stream_capturing():  # no event query or probe in a capture
            return 0, None
        if st is not None:
            ev, host = st
            if not ev.query():
                return 0, None
            self._defers[key] = nodefer = int(host[0]) == 0
            return (L.F_NO_GENERAL if nodefer else 0), None
        if len(self._defers) >= 64:
            self._defers.pop(next(iter(self._defers)))
        return 0, torch.full((1,), -1, dtype=torch.int32, device=self.device)

    def _probe_landed(self, key, probe) -> None:
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(probe, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._defers[key] = (ev, host)

    def _stats_ptr(self):
        return None if self.stats_buffer is None else self.stats_buffer.data_ptr()

    def _check_status(self, ws: torch.Tensor, key=None) -> None:
        """Raise what the kernel flagged in the workspace's status word (renders that can defer chains
        beyond the fast kernel's levels: a synchronisation). ``key``: a camera launch's identity
        (scene content, tile, cap; _tile_launch). The kernels are deterministic, so once a render of a
        key has come back clean an identical render cannot flag anything: later renders of that key
        skip the read-back and the host round trip (like _general_plan's probe; the status stays in
        the workspace untouched, clean)."""
        if self.max_bounces is None or self.max_bounces > L.FAST_MAX_BOUNCES:
            if key is not None and key in self._clean:
                return
            status = int(ws[:8].view(torch.int32)[1].item())
            if status == 0 and key is not None:
                if len(self._clean) >= 64:
                    self._clean.pop(next(iter(self._clean)))
                self._clean[key] = True
            if status:
                ws[4:8].zero_()  # sticky flags: clear for the next call
            if status & L.ST_BAD_SCENE:
                raise ValueError("the scene blob's header disagrees with n_spheres: nothing was rendered")
            if status & L.ST_STACK_OVERFLOW:
                raise RecursionError(f"maximum recursion depth exceeded (reflection chain > {L.UNBOUNDED_LEVELS} levels)")

    # ---------------------------------------------------------------- Renderer API
    def get_ray_directions(self, camera: Camera) -> HipCameraRays:
        """base.py:123-141 — lazy; see HipCameraRays."""
        camera_words((float(camera.position.x), float(camera.position.y), float(camera.position.z)),
                     camera.width, camera.height)  # validate now, like the reference would fail now
        return HipCameraRays(self, camera)

    def raytrace_scene(self, ray_origin: Vector3D, normalized_ray_direction: Vector3D, scene) -> HipRGBColor:
        """base.py:91-121 including every reflection level (shader.py:143-161)."""
        if isinstance(normalized_ray_direction, HipCameraRays) and normalized_ray_direction._data is None:
            cam = normalized_ray_direction.camera
            if _same_camera(cam, scene.camera) and _same_point(ray_origin, cam.position):
                return HipRGBColor.from_tensor(self.render_tile(scene))
        return HipRGBColor.from_tensor(self._trace(ray_origin, normalized_ray_direction, scene))

    def save_image(self, color, camera: Camera, output_path) -> None:
        """base.py:143-151: per channel (255*clip(c,0,1)).astype(uint8), reshaped (H, W), PNG."""
        hwc = self.quantize(color, camera)
        _write_png(hwc.cpu().numpy(), output_path)

    # ---------------------------------------------------------------- extensions
    def render(self, scene) -> HipRGBColor:
        """get_ray_directions + raytrace_scene of the scene camera (application.py:48-50), fused."""
        return HipRGBColor.from_tensor(self.render_tile(scene))

    @_on_device
    def render_tile(self, scene, row_block: int = 1, n_parts: int = 1, part: int = 0, out: str | None = None,
                    blob: torch.Tensor | None = None, n_spheres: int | None = None,
                    into: torch.Tensor | None = None, part_run: int = 1) -> torch.Tensor:
        """Render the interleaved row tile ``part`` of ``n_parts`` (row blocks of ``row_block``) of
        the scene camera's frame. Returns [3, rows*W] colour (``out=None``) or [rows, W, 3] uint8
        (``out="u8"``), rows in local order (python_ray_tracer_amd.tiling.tile_rows).

        ``into``: a contiguous device tensor of that shape and dtype to render into (a
        pre-allocated gather buffer) instead of a new one. ``blob``/``n_spheres``: an already
        packed device scene (checked against its header). ``part_run``: the run of parts
        part .. part + part_run - 1 as one tile (tiling.tile_rows with run)."""
        W = int(scene.camera.width)
        blob, n_spheres, rows, ws, flags, probe, key, order, cost = self._tile_launch(scene, row_block, n_parts, part,
                                                                                      blob, n_spheres, part_run)
        n = W * rows
        if out == "u8":
            shape, dtype, kind = (rows, W, 3), torch.uint8, L.OUT_U8_HWC
        else:
            shape, dtype, kind = (3, n), self.color_dtype, _OUT_KIND[self.color_dtype]
        if into is None:
            res = torch.empty(shape, dtype=dtype, device=self.device)
        else:
            if (tuple(into.shape) != shape or into.dtype != dtype or into.device != self.device
                    or not into.is_contiguous()):
                raise ValueError(f"into: need a contiguous {dtype} tensor of shape {shape} on {self.device}, got "
                                 f"{into.dtype} {tuple(into.shape)} on {into.device}")
            res = into
        L.check(self._lib.rtx_render_camera_sched(blob.data_ptr(), n_spheres, W, int(scene.camera.height), row_block,
                                                  n_parts, part, part_run, rows, self._bounces_arg, res.data_ptr(), kind,
                                                  ws.data_ptr(), ws.numel(), self._stats_ptr(), self._stream(), flags,
                                                  _ptr(probe), _ptr(order), _ptr(cost)), "rtx_render_camera")
        self._after_launch(key, probe, cost)
        self._check_status(ws, key if self.stats_buffer is None else None)  # (the full launch key only)
        return res

    def _after_launch(self, key, probe, cost) -> None:
        if probe is not None:
            self._probe_landed(key, probe)
        if cost is not None:
            self._cost_landed(key, cost)

    def _tile_launch(self, scene, row_block, n_parts, part, blob=None, n_spheres=None, part_run=1):
        """What a camera launch of one row tile needs: (blob, n_spheres, local rows, workspace, flags,
        probe, key, tile order, tile cost) — the scene's device blob (cached by content, or the
        caller's, checked), the general-kernel plan of a capped render (_general_plan) and the
        launch's dispatch order (_sched_plan)."""
        H = int(scene.camera.height)
        key = None
        if blob is None:
            key = scene_key(scene)
            blob, n_spheres = self._scene_entry(key)
        else:
            _check_blob(blob, n_spheres, self.device)
        rows = n_local_rows(H, row_block, n_parts, part, part_run)
        ws = self.workspace(int(scene.camera.width) * rows)
        flags, probe, order, cost = 0, None, None, None
        if key is not None and self.fast_textures and any(sp[2][0] == L.TEX_IMAGE for sp in key[0][0]):
            flags = L.F_IMAGES  # image-textured spheres shaded by the fast kernel, not deferred
        if key is not None and self.stats_buffer is None:
            key = (key, row_block, n_parts, part, part_run, self.max_bounces)
            # capped and uncapped alike (an uncapped render that defers nothing also skips the
            # continuation pass: unbounded C2 -4 us per frame)
            gflags, probe = self._general_plan(key)
            flags |= gflags
            if self.learn_tile_order:
                order, cost = self._sched_plan(key, int(scene.camera.width), rows, n_spheres)
        if torch.cuda.is_current_stream_capturing():
            # a captured launch keeps raw pointers to the blob, the workspace and the learnt order:
            # pin them for the renderer's life, so that a cache eviction (scene cache, workspace
            # growth, the 64-key order cache) cannot free memory a graph replay reads.
            # Keyed by address, so recapturing the same scene pins nothing new; release_graph_pins()
            # drops them once the caller has dropped its graphs
            self._graph_pins.update((t.data_ptr(), t) for t in (blob, ws, order) if t is not None)
        return blob, n_spheres, rows, ws, flags, probe, key, order, cost

    def release_graph_pins(self) -> int:
        """Forget the tensors pinned for graph replays (``_tile_launch``). Call it after dropping
        every CUDA graph captured from this renderer: a replay after it may read freed memory.
        Returns how many tensors were released."""
        n = len(self._graph_pins)
        self._graph_pins.clear()
        return n

    def _sched_plan(self, key, width, rows, n_spheres):
        """(tile_order, tile_cost) of a camera launch (rtx_render_camera_sched). The launch hands
        out its units (wave tiles of a persistent launch, block tiles otherwise) bottom-up; a few
        units with long reflection chains can then run alone at its end. The render is deterministic
        (same blob content, tile and cap: the same rays), so the first launch of a key records every
        unit's render time (tile_cost) and the units sorted by descending time (a device argsort
        enqueued right behind it: nothing waits, nothing crosses to the host) are the dispatch order
        of every later launch of the key. Output does not depend on the order."""
        if key in self._sched:  # the learnt order (None: a launch of a single unit)
            return self._sched[key], None
        if torch.cuda.is_current_stream_capturing():
            return None, None
        nt = ctypes.c_int64()
        L.check(self._lib.rtx_sched_tiles(width, rows, n_spheres, ctypes.byref(nt)), "rtx_sched_tiles")
        if nt.value <= 1:
            self._sched[key] = None  # nothing to order
            return None, None
        return None, torch.zeros(nt.value, dtype=torch.int32, device=self.device)

    def _cost_landed(self, key, cost) -> None:
        if len(self._sched) >= 64:
            self._sched.pop(next(iter(self._sched)))
        self._sched[key] = torch.argsort(cost, descending=True, stable=True).to(torch.int32)

    @_on_device
    def submit_tiles(self, plan, slot: int, scene, row_block: int, n_parts: int, part: int, frame,
                     part_run: int = 1) -> None:
        """One frame of a row-tiled plan (rtx_tiles_submit, distributed.TileGather): this rank's tile
        of ``scene`` rendered into the plan's slot, the RCCL gather to the root and, there, the
        assembly into ``frame`` (None on peers), all enqueued by one native call."""
        blob, n_spheres, rows, ws, flags, probe, key, order, cost = self._tile_launch(scene, row_block, n_parts, part,
                                                                                      part_run=part_run)
        L.check(self._lib.rtx_tiles_submit(plan, int(slot), blob.data_ptr(), n_spheres, self._bounces_arg,
                                           ws.data_ptr(), ws.numel(), flags, _ptr(probe), _ptr(order), _ptr(cost),
                                           _ptr(frame), self._stream()), "rtx_tiles_submit")
        self._after_launch(key, probe, cost)
        self._check_status(ws, key if self.stats_buffer is None else None)

    @_on_device
    def render_batch(self, scenes, out: str | None = None) -> torch.Tensor:
        """Whole frames of several scenes in ONE launch (rtx_render_frames).
        All scenes need the same camera size and sphere count; cameras, spheres and lights may
        differ (an animation). Returns [F, 3, W*H] colour (``out=None``) or [F, H, W, 3] uint8
        (``out="u8"``); frame f equals ``render_tile(scenes[f], out=out)``."""
        key, (blob, F, S, W, H) = self._batch_blob(scenes)
        n = W * H
        if out == "u8":
            res = torch.empty((F, H, W, 3), dtype=torch.uint8, device=self.device)
            kind = L.OUT_U8_HWC
        else:
            res = torch.empty((F, 3, n), dtype=self.color_dtype, device=self.device)
            kind = _OUT_KIND[self.color_dtype]
        ws = self.workspace(F * n)
        L.check(self._lib.rtx_render_frames(blob.data_ptr(), blob.shape[1], F, S, W, H, self._bounces_arg,
                                            res.data_ptr(), kind, ws.data_ptr(), ws.numel(), self._stats_ptr(),
                                            self._stream()), "rtx_render_frames")
        self._check_status(ws)
        return res

    def _batch_blob(self, scenes):
        """[F, L] device array of packed scenes (padded to the longest blob), cached by content."""
        keys = tuple(scene_key(sc) for sc in scenes)
        if not keys:
            raise ValueError("render_batch needs at least one scene")
        ck = ("batch", keys)
        hit = self._scene_cache.get(ck)
        if hit is None:
            (_, W, H) = keys[0][1]
            S = len(keys[0][0][0])
            for static, cam in keys:
                if cam[1:] != (W, H) or len(static[0]) != S:
                    raise ValueError("render_batch: every scene needs the same camera size and sphere count")
            blobs = [pack_key(*k) for k in keys]
            host = np.zeros((len(blobs), max(b.size for b in blobs)), dtype=np.float64)
            for f, b in enumerate(blobs):
                host[f, :b.size] = b
            dev = torch.from_numpy(host).pin_memory().to(self.device, non_blocking=True)
            hit = (dev, len(blobs), S, W, H)
            if len(self._scene_cache) >= 16:
                self._scene_cache.pop(next(iter(self._scene_cache)))
            self._scene_cache[ck] = hit
        return ck, hit

    @_on_device
    def _trace(self, ray_origin, dirs, scene) -> torch.Tensor:
        blob, S = self.scene_blob(scene)
        D = _as_vector(dirs).to_tensor(self.device)
        if D.dim() != 2:
            D = D.reshape(3, 1)
        n = D.shape[1]
        O = _as_vector(ray_origin).to_tensor(self.device, n)
        stride = 0 if O.dim() == 1 else n
        if stride and O.shape[1] != n:
            raise ValueError(f"origins ({O.shape[1]}) and directions ({n}) differ in length")
        res = torch.empty((3, n), dtype=self.color_dtype, device=self.device)
        ws = self.workspace(n)
        L.check(self._lib.rtx_trace_rays(blob.data_ptr(), S, O.data_ptr(), stride, D.data_ptr(), n,
                                         self._bounces_arg, res.data_ptr(), _OUT_KIND[self.color_dtype],
                                         ws.data_ptr(), ws.numel(), self._stats_ptr(), self._stream()),
                "rtx_trace_rays")
        self._check_status(ws)
        return res

    @_on_device
    def shade_hits(self, shape, scene, ray_origin, dirs, distance, shader=None) -> torch.Tensor:
        """NumpyShader.create of ``shader`` (default: ``shape``'s own) for rays hitting ``shape`` at
        ``distance`` (shader.py:63-112, rtx_shade_hits); the reflected rays are level 1 of this
        renderer's bounce cap and see the scene unchanged (another shape's shader shades only the
        level-0 hits, RTX_H_MAT0). Returns [3, n] colour."""
        si = next((k for k, s in enumerate(scene.shapes) if s is shape), None)
        if si is None:  # scene.shapes.index(shape) in _calculate_shadow (shader.py:126)
            raise ValueError("shape is not in scene.shapes")
        if shader is None or shader is getattr(shape, "shader", None):
            blob, S = self.scene_blob(scene)
        else:
            blob, S = self._override_blob(scene, si, shape, shader)
        D = _as_vector(dirs).to_tensor(self.device)
        if D.dim() != 2:
            D = D.reshape(3, 1)
        n = D.shape[1]
        O = _as_vector(ray_origin).to_tensor(self.device, n)
        stride = 0 if O.dim() == 1 else n
        if stride and O.shape[1] != n:
            raise ValueError(f"origins ({O.shape[1]}) and directions ({n}) differ in length")
        t = distance if _is_tensor(distance) else torch.from_numpy(np.asarray(distance, dtype=np.float64))
        t = t.to(device=self.device, dtype=torch.float64).reshape(-1)
        if t.numel() == 1 and n > 1:
            t = t.expand(n)
        t = t.contiguous()
        if t.numel() != n:
            raise ValueError(f"distance ({t.numel()}) and directions ({n}) differ in length")
        res = torch.empty((3, n), dtype=self.color_dtype, device=self.device)
        ws = self.workspace(n)
        L.check(self._lib.rtx_shade_hits(blob.data_ptr(), S, si, O.data_ptr(), stride, D.data_ptr(), t.data_ptr(), n,
                                         self._bounces_arg, res.data_ptr(), _OUT_KIND[self.color_dtype],
                                         ws.data_ptr(), ws.numel(), self._stats_ptr(), self._stream()),
                "rtx_shade_hits")
        self._check_status(ws)
        return res

    def _override_blob(self, scene, si, shape, shader):
        """The scene blob with a level-0 material record for ``shader`` (scene_pack.pack_override),
        cached by content like scene_blob."""
        import types

        from .scene_pack import _shape_fields, pack_override

        pos = getattr(shape, "position", None) or getattr(shape, "center", None)
        key = ("mat0", scene_key(scene), si,
               _shape_fields(types.SimpleNamespace(position=pos, radius=shape.radius, shader=shader)))
        hit = self._scene_cache.get(key)
        if hit is None:
            blob = pack_override(scene, shape, shader)
            hit = (torch.from_numpy(blob).pin_memory().to(self.device, non_blocking=True), int(blob[L.H_NSPH]))
            if len(self._scene_cache) >= 16:
                self._scene_cache.pop(next(iter(self._scene_cache)))
            self._scene_cache[key] = hit
        return hit

    @_on_device
    def _ray_directions(self, camera: Camera) -> torch.Tensor:
        # a camera-only blob: no shapes needed for ray generation
        pos = (float(camera.position.x), float(camera.position.y), float(camera.position.z))
        blob = np.zeros(L.HDR_WORDS, dtype=np.float64)
        cw = camera_words(pos, camera.width, camera.height)
        blob[L.H_CAM:L.H_CAM + 3] = pos
        blob[L.H_XSTART], blob[L.H_XSTEP], blob[L.H_XSTOP], blob[L.H_XFIX] = cw["xs"]
        blob[L.H_YSTART], blob[L.H_YSTEP], blob[L.H_YSTOP], blob[L.H_YFIX] = cw["ys"]
        blob[L.H_VZ], blob[L.H_VZ2] = cw["vz"], cw["vz2"]
        dev_blob = torch.from_numpy(blob).to(self.device)
        W, H = int(camera.width), int(camera.height)
        out = torch.empty((3, W * H), dtype=torch.float64, device=self.device)
        L.check(self._lib.rtx_ray_directions(dev_blob.data_ptr(), W, H, 1, 1, 0, H, out.data_ptr(), self._stream()),
                "rtx_ray_directions")
        return out

    @_on_device
    def quantize(self, color, camera: Camera) -> torch.Tensor:
        """Device-side ``(255*clip(c,0,1)).astype(uint8)`` -> [H, W, 3] uint8 (base.py:145-149)."""
        W, H = int(camera.width), int(camera.height)
        t = color.data if isinstance(color, HipRGBColor) and hasattr(color, "data") else _as_vector(color).to_tensor(self.device)
        if t.dim() == 1:
            t = t.reshape(3, 1)
        if t.dtype not in _OUT_KIND:
            t = t.to(torch.float64)
        # a colour assembled on the host (a gloo gather) or built by the caller from CPU tensors:
        # the kernel reads device memory only
        t = t.to(self.device).contiguous()
        n = t.shape[1]
        if n != W * H:
            # np.reshape in save_image (base.py:147)
            raise ValueError(f"cannot reshape array of size {n} into shape ({H},{W})")
        out = torch.empty((H, W, 3), dtype=torch.uint8, device=self.device)
        L.check(self._lib.rtx_quantize_u8(t.data_ptr(), _OUT_KIND[t.dtype], n, out.data_ptr(), self._stream()),
                "rtx_quantize_u8")
        return out

    @_on_device
    def assemble_rows(self, tiles: torch.Tensor, width: int, height: int, row_block: int,
                      out: str | None = None, root_run: int = 1, run: int = 1) -> torch.Tensor:
        """Frame from gathered row tiles (rtx_assemble_rows, the device un-permute of the
        multi-GPU path): ``tiles`` is [n_parts, part_len], part p holding render_tile(...,
        row_block, n_parts, p, out) flattened at its start. Returns what a whole-frame
        render_tile returns: [3, H*W] colour or [H, W, 3] uint8 (``out="u8"``). ``root_run`` /
        ``run``: tile r is the run of parts of rank r (tiling.runs)."""
        P = int(tiles.shape[0])
        if tiles.device != self.device or not tiles.is_contiguous():
            tiles = tiles.to(self.device).contiguous()
        if out == "u8":
            kind, res = L.OUT_U8_HWC, torch.empty((height, width, 3), dtype=torch.uint8, device=self.device)
        else:
            kind = _OUT_KIND[tiles.dtype]
            res = torch.empty((3, height * width), dtype=tiles.dtype, device=self.device)
        stride = tiles.stride(0) * tiles.element_size()
        L.check(self._lib.rtx_assemble_runs(tiles.data_ptr(), stride, P, root_run, run, width, height, row_block, kind,
                                            res.data_ptr(), self._stream()), "rtx_assemble_runs")
        return res

    def stats(self) -> dict:
        """Per-level counters accumulated since construction / reset_stats (synchronises)."""
        if self.stats_buffer is None:
            raise RuntimeError("construct HipRenderer(collect_stats=True) to count rays")
        s = self.stats_buffer.cpu().tolist()
        rays = s[L.S_RAYS:L.S_RAYS + L.S_LEVELS]
        hits = s[L.S_HITS:L.S_HITS + L.S_LEVELS]
        last = max([i + 1 for i, v in enumerate(rays) if v] or [0])
        return {"pixels": s[L.S_PIXELS], "deferred": s[L.S_DEFERRED], "ties": s[L.S_TIES],
                "sphere_tests": s[L.S_TESTS], "node_tests": s[L.S_NODES],
                "sphere_tests_reflected": s[L.S_TESTS1], "node_tests_reflected": s[L.S_NODES1],
                "beam_searches": s[L.S_BEAMW], "box_tests": s[L.S_BOXES], "beam_tests": s[L.S_BEAMT],
                "rays": rays[:last], "hits": hits[:last],
                "waves_traced": s[L.S_WTRACE:L.S_WTRACE + last], "waves_shaded": s[L.S_WSHADE:L.S_WSHADE + last]}

    def reset_stats(self) -> None:
        if self.stats_buffer is not None:
            self.stats_buffer.zero_()


def _ptr(t):
    return None if t is None else t.data_ptr()


def _resolve_device(device) -> torch.device:
    """The renderer's device with an explicit index: None and an index-less "cuda" mean the
    current device at construction (``_on_device`` switches to ``device.index``, which must not be
    None). Anything but a ROCm device is refused: there is no CPU path."""
    d = torch.device("cuda") if device is None else torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"HipRenderer renders on a ROCm device ('cuda[:N]'), got {d}")
    return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())


def _as_vector(v) -> HipVector3D:
    if isinstance(v, HipVector3D):
        return v
    if isinstance(v, torch.Tensor) and v.dim() >= 1 and v.shape[0] == 3:
        return HipVector3D(v[0], v[1], v[2])
    if hasattr(v, "x") and hasattr(v, "y") and hasattr(v, "z"):
        return HipVector3D(v.x, v.y, v.z)
    raise TypeError(f"expected a 3-vector, got {type(v).__name__}")


def _check_blob(blob: torch.Tensor, n_spheres, device) -> None:
    """A caller-supplied packed scene: float64, contiguous, on the renderer's device, and its
    header's sphere count equal to ``n_spheres`` (the kernels size the LDS table and every sphere
    loop by it). Reads the header back: one small synchronous copy."""
    if not isinstance(blob, torch.Tensor) or blob.dtype != torch.float64 or blob.dim() != 1 or not blob.is_contiguous():
        raise ValueError("blob: need a contiguous 1-D float64 tensor (scene_pack.pack_scene)")
    if blob.device != torch.device(device):
        raise ValueError(f"blob is on {blob.device}, the renderer on {device}")
    if blob.numel() < L.HDR_WORDS:
        raise ValueError("blob shorter than the scene header")
    hdr = blob[:L.H_NSPH + 1].cpu().tolist()
    if hdr[L.H_MAGIC] != L.MAGIC:
        raise ValueError("blob is not a packed scene (bad magic)")
    if n_spheres is None or int(hdr[L.H_NSPH]) != int(n_spheres):
        raise ValueError(f"n_spheres={n_spheres!r} but the blob holds {int(hdr[L.H_NSPH])} spheres")
    need = L.HDR_WORDS + int(hdr[L.H_NSPH]) * (L.GEOM_WORDS + L.MAT_WORDS)
    if blob.numel() < need:
        raise ValueError(f"blob too short for {int(hdr[L.H_NSPH])} spheres ({blob.numel()} < {need} words)")


def _same_point(a, b) -> bool:
    try:
        return all(np.ndim(u) == 0 and float(u) == float(w) for u, w in zip(_as_vector(a).components(),
                                                                            _as_vector(b).components()))
    except TypeError:
        return False


def _same_camera(a: Camera, b: Camera) -> bool:
    return a is b or (int(a.width) == int(b.width) and int(a.height) == int(b.height)
                      and _same_point(a.position, b.position))


def _write_png(hwc: np.ndarray, output_path) -> None:
    from PIL import Image

    # base.py:145-151 builds three "L" images and merges them into "RGB": same pixels.
    img = Image.fromarray(np.ascontiguousarray(hwc, dtype=np.uint8))
    if hasattr(output_path, "write"):  # file object: PNG (a path's extension picks the format, like PIL in base.py:151)
        img.save(output_path, format="PNG")
        return
    # written to a temporary name and renamed, so an interrupted write never leaves a truncated
    # file under the final name (render_frames treats an existing file as finished)
    path = Path(output_path)
    tmp = path.with_name(path.name + ".tmp")
    img.save(tmp, format=Image.registered_extensions().get(path.suffix.lower(), "PNG"))
    os.replace(tmp, path)
