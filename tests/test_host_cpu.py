"""CPU-only tests of the host layer: C-ABI library exports, scene packing, tiling, error behaviour.
No compute call reaches the GPU here."""

import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import numpy_oracle as O
from python_ray_tracer_amd import scenes, tiling
from python_ray_tracer_amd.infrastructure.hip import _lib as L
from python_ray_tracer_amd.infrastructure.hip import scene_pack
from tests.conftest import REPO
from tests.specs import HUGE_LAYOUTS, huge_tail_spec


def _header_functions():
    text = (REPO / "include" / "rtx_hip.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(rtx_\w+)\(", text, re.M)))


def test_library_exports_every_header_symbol():
    lib = L.load()
    declared = _header_functions()
    assert set(declared) == set(L.EXPORTS), declared
    for name in declared:
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_library_links_both_units():
    """librtx_hip.so is two translation units (csrc/rtx_kernels.hip + csrc/rtx_small.hip, the
    small-scene kernels): the launch entry of the small unit is defined inside the library (a
    one-unit build would leave it undefined, found only at the first small-scene render) and hidden."""
    L.load()
    so = str(REPO / "python_ray_tracer_amd" / "librtx_hip.so")
    import shutil

    nm = shutil.which("nm") or shutil.which("llvm-nm")
    if nm is None:
        pytest.skip("no nm on PATH")
    undefined = subprocess.run([nm, "-D", "--undefined-only", so], check=True, capture_output=True, text=True).stdout
    assert "rtx_launch_small" not in undefined
    local = subprocess.run([nm, "-C", so], check=True, capture_output=True, text=True).stdout
    assert re.search(r"^\w+ t rtx_launch_small\(", local, re.M), "rtx_launch_small: not a hidden definition"
    dynamic = subprocess.run([nm, "-D", so], check=True, capture_output=True, text=True).stdout
    assert "rtx_launch_small" not in dynamic


def test_abi_layout_matches_header():
    text = (REPO / "include" / "rtx_hip.h").read_text()

    def const(name):
        m = re.search(rf"\b{name}\s*=\s*(-?\d+)", text) or re.search(rf"#define\s+{name}\s+\(?(-?[\d.]+)", text)
        return float(m.group(1))

    assert const("RTX_HDR_WORDS") == L.HDR_WORDS
    assert const("RTX_GEOM_WORDS") == L.GEOM_WORDS
    assert const("RTX_MAT_WORDS") == L.MAT_WORDS
    assert const("RTX_S_WORDS") == L.S_WORDS
    assert const("RTX_S_BOXES") == L.S_BOXES
    assert const("RTX_S_BEAMT") == L.S_BEAMT
    assert const("RTX_H_CAMOO") == L.H_CAMOO
    assert const("RTX_M_TFIOR") == L.M_TFIOR
    assert const("RTX_G_C0") == L.G_C0
    assert const("RTX_H_TAME") == L.H_TAME
    assert const("RTX_H_SHGRID") == L.H_SHGRID
    assert const("RTX_H_SINRED") == L.H_SINRED
    assert const("RTX_H_NBEAM") == L.H_NBEAM
    assert const("RTX_H_SBOX") == L.H_SBOX
    assert const("RTX_MAGIC") == L.MAGIC
    assert const("RTX_UNBOUNDED_LEVELS") == L.UNBOUNDED_LEVELS
    lay = (ctypes.c_int * 8)()
    assert L.load().rtx_abi_version(lay, 8) == L.ABI_VERSION


def test_workspace_bytes_and_error_paths():
    lib = L.load()
    assert lib.rtx_workspace_bytes(1920 * 1080, 3) >= L.WS_HDR_BYTES + 8 * 1920 * 1080
    # argument validation happens before any HIP call: no GPU needed
    rc = lib.rtx_render_camera(None, 3, 16, 16, 1, 1, 0, 16, 3, None, 0, None, 0, None, None)
    assert rc == -1 and b"null" in lib.rtx_last_error()
    rc = lib.rtx_render_camera(None, 3, 16, 16, 1, 2, 5, 16, 3, None, 0, None, 0, None, None)
    assert rc == -1 and b"geometry" in lib.rtx_last_error()
    rc = lib.rtx_render_frames(None, 0, 2, 3, 16, 16, 3, None, 0, None, 0, None, None)
    assert rc == -1 and b"scene_stride" in lib.rtx_last_error()
    assert lib.rtx_render_frames(None, 64, -1, 3, 16, 16, 3, None, 0, None, 0, None, None) == -1
    assert lib.rtx_render_frames(None, 64, 0, 3, 16, 16, 3, None, 0, None, 0, None, None) == 0  # nothing to do
    assert lib.rtx_render_frames(None, 64, 70000, 3, 16, 16, 3, None, 0, None, 0, None, None) == -1
    assert lib.rtx_quantize_u8(None, 0, 10, None, None) == -1
    assert lib.rtx_sphere_intersect(None, None, 0, None, 5, None, None) == -1


def test_sched_and_tiles_entry_points_validate_on_host():
    """The dispatch-order and row-tiled-frame entry points (round 4): unit counts of a launch, and
    the argument checks that run before any HIP or RCCL call (no GPU needed)."""
    lib = L.load()
    text = (REPO / "include" / "rtx_hip.h").read_text()
    for name, val in (("RTX_TILES_LOOPBACK", L.TILES_LOOPBACK), ("RTX_TILES_ROWS", L.TILES_ROWS),
                      ("RTX_TILES_TIMED", L.TILES_TIMED),
                      ("RTX_F_RESERVE_SHIFT", L.F_RESERVE_SHIFT), ("RTX_F_IMAGES", L.F_IMAGES), ("RTX_TILES_MAX_SLOTS", L.TILES_MAX_SLOTS)):
        assert int(re.search(rf"#define\s+{name}\s+(\d+)", text).group(1)) == val, name
    n = ctypes.c_int64()
    # a persistent launch (>= 32 spheres) hands out 8x8 wave tiles
    assert lib.rtx_sched_tiles(7680, 4320, 65, ctypes.byref(n)) == 0 and n.value == 960 * 540
    # below 8 spheres: one-wave blocks of 16x4 pixels
    assert lib.rtx_sched_tiles(1920, 1080, 3, ctypes.byref(n)) == 0 and n.value == 120 * 270
    # 8..31 spheres: block tiles of 4x1 waves of 8x8 pixels (32 x 8)
    assert lib.rtx_sched_tiles(3840, 2160, 17, ctypes.byref(n)) == 0 and n.value == 120 * 270
    assert lib.rtx_sched_tiles(1920, 0, 3, ctypes.byref(n)) == 0 and n.value == 0
    # unknown flag bits are refused before anything is launched
    rc = lib.rtx_render_camera_sched(None, 3, 16, 16, 1, 1, 0, 1, 16, 3, None, 0, None, 0, None, None, 1 << 20, None,
                                     None, None)
    assert rc == -1 and b"flags" in lib.rtx_last_error()
    # a run of parts past the interleave, an empty run, more local rows than the run owns
    for part, run, rows in ((3, 2, 4), (0, 0, 4), (1, 2, 9)):
        rc = lib.rtx_render_camera_sched(None, 3, 16, 16, 2, 4, part, run, rows, 3, None, 0, None, 0, None, None, 0,
                                         None, None, None)
        assert rc == -1 and b"geometry" in lib.rtx_last_error(), (part, run, rows)
    plan = ctypes.c_void_p()
    ptrs = (ctypes.c_void_p * 2)(1, 1)
    # a gathering plan needs a communicator (RTX_E_COMM); RTX_TILES_ROWS needs uint8 frames
    assert lib.rtx_tiles_create(None, 2, 0, 0, 64, 64, 8, L.OUT_U8_HWC, 2, ptrs, ptrs, 4096, 1, 1, 0,
                                ctypes.byref(plan)) == -4
    assert lib.rtx_tiles_create(None, 2, 0, 0, 64, 64, 8, L.OUT_F32_SOA, 2, ptrs, ptrs, 8192, 1, 1, L.TILES_ROWS,
                                ctypes.byref(plan)) == -1
    assert lib.rtx_tiles_create(None, 1, 0, 0, 64, 64, 8, L.OUT_U8_HWC, 9, None, None, 16, 1, 1, 0,
                                ctypes.byref(plan)) == -1
    assert lib.rtx_tiles_create(None, 1, 0, 0, 64, 64, 8, L.OUT_U8_HWC, 2, None, None, 16, 1, 1, 1 << 20,
                                ctypes.byref(plan)) == -1
    # unequal shares: rank 0 must be the root, and a one-rank plan has one share
    assert lib.rtx_tiles_create(None, 1, 0, 0, 64, 64, 8, L.OUT_U8_HWC, 2, None, None, 16, 1, 2, 0,
                                ctypes.byref(plan)) == -1
    assert plan.value is None
    assert lib.rtx_tiles_submit(None, 0, None, 3, 3, None, 0, 0, None, None, None, None, None) == -1
    assert lib.rtx_tiles_destroy(None) == 0
    f1, f2 = ctypes.c_float(), ctypes.c_float()
    assert lib.rtx_tiles_timing(None, 0, ctypes.byref(f1), ctypes.byref(f2)) == -1


def test_pack_matches_reference_expressions():
    spec = scenes.readme_spec(160, 90)
    sc = scenes.build_scene(spec)  # HipSphere & co. need no GPU to construct
    blob = scene_pack.pack_scene(sc)
    S = len(spec["spheres"])
    assert blob[L.H_NSPH] == S and blob[L.H_MAGIC] == L.MAGIC
    geo = blob[L.HDR_WORDS:L.HDR_WORDS + S * L.GEOM_WORDS].reshape(S, -1)
    mat = blob[L.HDR_WORDS + S * L.GEOM_WORDS:L.HDR_WORDS + S * (L.GEOM_WORDS + L.MAT_WORDS)].reshape(S, -1)
    # level-0 "c" of shape.py:35-37 equals the oracle's scalar evaluation
    for s, sp in enumerate(spec["spheres"]):
        cx, cy, cz = sp["center"]
        ox, oy, oz = spec["camera"]["position"]
        c = ((cx * cx + cy * cy) + cz * cz) + ((ox * ox + oy * oy) + oz * oz) - 2 * ((cx * ox + cy * oy) + cz * oz) \
            - (sp["radius"] * sp["radius"])
        assert geo[s, L.G_C0] == c
        assert geo[s, L.G_INVR] == 1.0 / sp["radius"]
        r = sp["shader"]["specular_roughness"]
        assert mat[s, L.M_A2] == (r**2) ** 2
        assert mat[s, L.M_F0] == ((1.5 - 1) / (1.5 + 1)) ** 2
    assert mat[2, L.M_TEX] == 1.0 and mat[0, L.M_TEX] == 0.0
    # linspace parameters reproduce np.linspace exactly
    for W, H in ((1, 1), (2, 3), (7, 5), (960, 540), (1920, 1080), (7680, 4320)):
        cw = scene_pack.camera_words((0.0, 0.2, -2.0), W, H)
        ar = float(W) / H
        for (start, step, stop, fix), want in ((cw["xs"], np.linspace(-1, 1, W)),
                                               (cw["ys"], np.linspace(1 / ar + 0.25, -1 / ar + 0.25, H))):
            i = np.arange(len(want), dtype=np.float64)
            got = i * step + start
            if fix:
                got[-1] = stop
            assert np.array_equal(got, want), (W, H)


@pytest.mark.parametrize("n", [0, 7, 8, 16, 64, 200])
def test_culling_tree_invariants(n):
    """Packer's box tree: every small sphere in exactly one leaf, leaves' boxes contain their
    spheres (and every ancestor's box contains them), skip links close each subtree, margins are
    positive, huge spheres are in the always-tested prefix."""
    spec = scenes.random_spec(n, 3, 64, 36)
    blob = scene_pack.pack_scene(scenes.build_scene(spec))
    S = n + 1
    nn = int(blob[L.H_NNODES])
    if S < scene_pack.BVH_MIN_SPHERES:
        assert nn == 0
        return
    nodes = blob[int(blob[L.H_NODES]):int(blob[L.H_NODES]) + nn * L.NODE_WORDS].reshape(nn, L.NODE_WORDS)
    cg = blob[int(blob[L.H_CGEO]):int(blob[L.H_CGEO]) + S * L.GEOM_WORDS].reshape(S, L.GEOM_WORDS)
    geo = blob[L.HDR_WORDS:L.HDR_WORDS + S * L.GEOM_WORDS].reshape(S, L.GEOM_WORDS)
    nal = int(blob[L.H_NALWAYS])
    assert sorted(cg[:, L.G_IDX].astype(int).tolist()) == list(range(S))
    assert nal == 1 and int(cg[0, L.G_IDX]) == n  # the ground sphere (appended last) is always tested
    assert int(blob[L.H_NBEAM]) == n  # ... and is the scene's huge tail (no frustum or beam test)
    for k in range(S):  # the culled list carries the same geometry words
        s = int(cg[k, L.G_IDX])
        assert np.array_equal(cg[k, :L.G_IDX], geo[s, :L.G_IDX])
    covered = []

    def walk(i, ancestors):
        node = nodes[i]
        end = int(node[L.N_SKIP])
        assert i < end <= nn
        if node[L.N_COUNT] > 0:
            for k in range(int(node[L.N_FIRST]), int(node[L.N_FIRST] + node[L.N_COUNT])):
                covered.append(k)
                s = int(cg[k, L.G_IDX])
                r = np.sqrt(geo[s, L.G_RR])
                for a in ancestors + [node]:
                    assert np.all(a[L.N_LOX:L.N_LOZ + 1] <= geo[s, :3] - r)
                    assert np.all(geo[s, :3] + r <= a[L.N_HIX:L.N_HIZ + 1])
                    assert a[L.N_MARGIN] >= 2e-7
            assert end == i + 1
            return end
        j = i + 1
        while j < end:
            j = walk(j, ancestors + [node])
        assert j == end
        return end

    assert walk(0, []) == nn
    assert sorted(covered) == list(range(nal, S))


def test_pack_error_behaviour():
    from python_ray_tracer_amd.domain import Camera, DomeLight, Scene3D
    from python_ray_tracer_amd.infrastructure.hip import HipRGBColor, HipVector3D

    spec = scenes.readme_spec(8, 8)
    sc = scenes.build_scene(spec)
    with pytest.raises(TypeError):  # reduce() of empty iterable (base.py:98)
        scene_pack.pack_scene(Scene3D([], sc.lights, sc.camera))
    with pytest.raises(IndexError):  # scene.lights[0] (shader.py:75)
        scene_pack.pack_scene(Scene3D(sc.shapes, [], sc.camera))
    with pytest.raises(AttributeError):  # DomeLight has no position (shader.py:75)
        scene_pack.pack_scene(Scene3D(sc.shapes, [DomeLight(0.1, HipRGBColor(1, 1, 1))], sc.camera))
    with pytest.raises(ValueError):
        scene_pack.pack_scene(Scene3D(sc.shapes, sc.lights, Camera(HipVector3D(0, 0, -2), 0, 5)))


@pytest.mark.parametrize("H,rb,P", [(1080, 8, 8), (1080, 8, 3), (13, 4, 3), (5, 8, 2), (4320, 8, 8), (7, 1, 7)])
def test_tiling_partition(H, rb, P):
    seen = np.concatenate([tiling.tile_rows(H, rb, P, p) for p in range(P)])
    assert np.array_equal(np.sort(seen), np.arange(H))
    for p in range(P):
        r = tiling.tile_rows(H, rb, P, p)
        assert len(r) == tiling.n_local_rows(H, rb, P, p)
        assert np.all(np.diff(r) > 0)
    assert tiling.max_local_rows(H, rb, P) == max(tiling.n_local_rows(H, rb, P, p) for p in range(P))
    # assemble inverts the split, from the flat gather buffers (colour and uint8 layouts)
    W = 3
    frame = np.arange(3 * H * W, dtype=np.float64).reshape(3, H, W)
    L = tiling.part_len(H, W, rb, P, 8)
    assert L >= 3 * tiling.max_local_rows(H, rb, P) * W and (L * 8) % 16 == 0
    tiles = np.full((P, L), -1.0)
    hwc = (frame.reshape(3, H * W).T.reshape(H, W, 3) % 251).astype(np.uint8)
    L8 = tiling.part_len(H, W, rb, P, 1, "u8")
    tiles8 = np.zeros((P, L8), dtype=np.uint8)
    for p in range(P):
        r = tiling.tile_rows(H, rb, P, p)
        assert tiling.tile_shape(H, W, rb, P, p) == (3, len(r) * W)
        tiles[p, :3 * len(r) * W] = frame[:, r].reshape(-1)
        tiles8[p, :3 * len(r) * W] = hwc[r].reshape(-1)
    assert np.array_equal(tiling.assemble(tiles, H, W, rb), frame.reshape(3, H * W))
    assert np.array_equal(tiling.assemble(torch.from_numpy(tiles), H, W, rb).numpy(), frame.reshape(3, H * W))
    assert np.array_equal(tiling.assemble(tiles8, H, W, rb, "u8"), hwc)


def test_hip_renderer_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    with pytest.raises(RuntimeError, match="no CPU path"):
        HipRenderer()


def test_random_scene_generator_is_seeded():
    a = scenes.random_spec(16, 0)
    b = scenes.random_spec(16, 0)
    assert a == b and len(a["spheres"]) == 17
    for s in a["spheres"][:-1]:
        assert abs(s["center"][1] - (s["radius"] - 0.5)) < 1e-15
    sc = O.scene_from_spec(a)
    assert sc.spheres[-1].checker and sc.light_pos == (-2, 4, -1)


def test_render_frames_batches_by_shape(tmp_path):
    """application.render_frames: with a renderer that has render_batch, consecutive frames of one
    camera size and sphere count go out in batches of at most `batch`; frames whose PNG exists are
    skipped (resumable); every frame's colour comes back under its index."""
    from python_ray_tracer_amd.application import render_frames

    calls = []

    class FakeBatchRenderer:
        def render_batch(self, scenes_):
            calls.append([int(s.camera.width) for s in scenes_])
            return torch.stack([torch.full((3, int(s.camera.width) * int(s.camera.height)), float(len(s.shapes)))
                                for s in scenes_])

        def save_image(self, color, camera, path):
            path.write_bytes(b"png")

    def frame(w, n):
        return scenes.build_scene(scenes.random_spec(n, 0, w, 4))

    frames = [frame(8, 3), frame(8, 3), frame(8, 3), frame(6, 3), frame(6, 3), frame(8, 5), frame(8, 5)]
    (tmp_path / "frame_0001.png").write_bytes(b"old")
    out = render_frames(frames, FakeBatchRenderer(), tmp_path, batch=2)
    assert sorted(out) == [0, 2, 3, 4, 5, 6]
    assert calls == [[8, 8], [6, 6], [8, 8]]  # (0, 2), (3, 4), (5, 6): shape changes split batches
    assert float(out[5].data[0, 0]) == 6.0  # 5 random spheres + ground
    assert (tmp_path / "frame_0001.png").read_bytes() == b"old"


@pytest.mark.parametrize("backend", ["numpy", "torch"])
def test_vector_algebra_matches_reference_expressions(backend):
    """HipVector3D (reference NumpyVector3D, base.py:28-79): dot = (xx + yy) + zz, abs = squared
    norm, norm = v * (1 / where(|v| == 0, 1, |v|)), extract = np.extract, place = scatter into
    zeros; with NumPy or (CPU) torch components, bit for bit."""
    from python_ray_tracer_amd.infrastructure.hip import HipVector3D

    rng = np.random.default_rng(5)
    a = rng.normal(size=(3, 33))
    b = rng.normal(size=(3, 33))
    a[:, 7] = 0.0  # a zero vector: norm keeps it zero
    cond = rng.random(33) < 0.4
    wrap = (lambda x: torch.from_numpy(x)) if backend == "torch" else (lambda x: x)
    va, vb = HipVector3D(*map(wrap, a)), HipVector3D(*map(wrap, b))

    def arr(x):
        return x.numpy() if isinstance(x, torch.Tensor) else np.asarray(x)

    dot = (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]
    assert np.array_equal(arr(va.dot(vb)), dot)
    assert np.array_equal(arr(abs(va)), (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2])
    for got, want in ((va * vb, a * b), (va * 2.5, a * 2.5), (va + vb, a + b), (va - vb, a - b), (-va, -a),
                      (va / 3.0, a / 3.0)):
        assert all(np.array_equal(arr(g), w) for g, w in zip(got.components(), want))
    mag = np.sqrt((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2])
    want = a * (1.0 / np.where(mag == 0, 1, mag))
    assert all(np.array_equal(arr(g), w) for g, w in zip(va.norm().components(), want))
    ex = va.extract(wrap(cond))
    assert all(np.array_equal(arr(g), np.extract(cond, w)) for g, w in zip(ex.components(), a))
    back = ex.place(wrap(cond))
    for g, w in zip(back.components(), a):
        z = np.zeros(33)
        np.place(z, cond, np.extract(cond, w))
        assert np.array_equal(arr(g), z)


def test_torch_ops_registered_and_checked_on_host():
    """torch.ops.rt (csrc/rt_ops.cpp, TORCH_LIBRARY over the C ABI) loads without a GPU; its size
    query equals the C ABI's; host tensors, wrong dtypes and short workspaces raise RuntimeError
    (TORCH_CHECK) before anything is launched."""
    import python_ray_tracer_amd.ops as ops
    from python_ray_tracer_amd.infrastructure.hip import _lib as L

    lib = L.load()
    for name in ops.OPS:
        assert hasattr(torch.ops.rt, name), name
    for n, B in ((1, 0), (2073600, 3), (33177600, 5), (1000, -1)):
        assert torch.ops.rt.workspace_bytes(n, B) == lib.rtx_workspace_bytes(n, B)
    blob = torch.zeros(200, dtype=torch.float64)
    ws = torch.zeros(64, dtype=torch.uint8)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.render_tile(blob, 3, 8, 8, 1, 1, 0, 3, 0, ws)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.trace(blob, 3, torch.zeros(3, dtype=torch.float64), torch.zeros(3, 5, dtype=torch.float64), 3, 0,
                           ws)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.intersect(torch.zeros(8, dtype=torch.float64), torch.zeros(3, dtype=torch.float64),
                               torch.zeros(3, 5, dtype=torch.float64))
    with pytest.raises(RuntimeError):
        torch.ops.rt.quantize_u8(torch.zeros(3, 4))
    with pytest.raises(RuntimeError):
        torch.ops.rt.assemble_rows(torch.zeros(2, 64, dtype=torch.uint8), 4, 4, 1, 2)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.render_frames(torch.zeros(2, 200, dtype=torch.float64), 3, 8, 8, 3, 0, ws)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.shade_hits(blob, 3, 0, torch.zeros(3, dtype=torch.float64), torch.zeros(3, 5, dtype=torch.float64),
                                torch.zeros(5, dtype=torch.float64), 3, 0, ws)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.status(ws)


def test_tiles_ops_schema_and_host_checks():
    """The native row-tiled frame through the op surface (rtx_tiles_* had no op): the
    communicator and plan ops exist with int64 handles, mutate the workspace and frame they are given,
    and refuse bad arguments on the host before anything is created or launched."""
    import python_ray_tracer_amd.ops  # noqa: F401

    sch = {n: str(getattr(torch.ops.rt, n).default._schema) for n in
           ("comm_unique_id", "comm_init", "comm_destroy", "tiles_create", "tiles_submit", "tiles_finish",
            "tiles_destroy")}
    assert sch["comm_unique_id"].endswith("-> Tensor")
    assert "Tensor unique_id, int world, int rank, int device=-1, int max_ctas=0) -> int" in sch["comm_init"]
    assert "int slots, Tensor[] send, Tensor[] recv, int part_bytes, int root_run=1, int run=1, int flags=0" \
        in sch["tiles_create"] and sch["tiles_create"].endswith("-> int")
    assert "Tensor(a!) workspace, Tensor(b!)? frame=None, int flags=0) -> ()" in sch["tiles_submit"]
    assert "int plan, int slot, int device" in sch["tiles_finish"]
    with pytest.raises(RuntimeError, match="unique_id"):
        torch.ops.rt.comm_init(torch.zeros(64, dtype=torch.uint8), 1, 0)
    with pytest.raises(RuntimeError, match="slots"):
        torch.ops.rt.tiles_create(0, 1, 0, 0, 8, 8, 1, 2, 0, [], [], 256)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.tiles_create(0, 2, 1, 0, 8, 8, 1, 2, 1, [torch.zeros(256, dtype=torch.uint8)], [], 256)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        torch.ops.rt.tiles_submit(0, 0, torch.zeros(200, dtype=torch.float64), 3, 3, torch.zeros(64, dtype=torch.uint8))


def test_torch_ops_schema_and_fake_kernels():
    """The render ops declare their workspace and stats as mutated (Tensor(a!), Tensor(b!)?) and
    carry a check flag; every op has a Meta kernel returning the output a GPU call returns, so the
    surface traces under FakeTensor (torch.compile) without a GPU."""
    import python_ray_tracer_amd.ops  # noqa: F401

    for name in ("render_tile", "render_frames", "trace", "shade_hits"):
        s = str(getattr(torch.ops.rt, name).default._schema)
        assert "Tensor(a!) workspace" in s and "Tensor(b!)? stats=None" in s and "bool check=True" in s, s
    meta = {"device": "meta"}
    blob = torch.empty(64 + 3 * 32, dtype=torch.float64, **meta)
    ws = torch.empty(1 << 20, dtype=torch.uint8, **meta)
    st = torch.empty(L.S_WORDS, dtype=torch.int64, **meta)
    assert torch.ops.rt.render_tile(blob, 3, 20, 17, 1, 1, 0, 3, 0, ws, st).shape == (3, 340)
    out = torch.ops.rt.render_tile(blob, 3, 20, 17, 4, 3, 1, 3, 2, ws)  # rows 4-7 and 16: 5 rows
    assert out.shape == (5, 20, 3) and out.dtype == torch.uint8
    assert torch.ops.rt.render_tile(blob, 3, 20, 17, 1, 1, 0, 3, 1, ws).dtype == torch.float64
    frames = torch.empty(4, 160, dtype=torch.float64, **meta)
    assert torch.ops.rt.render_frames(frames, 3, 20, 17, 3, 2, ws).shape == (4, 17, 20, 3)
    assert torch.ops.rt.render_frames(frames, 3, 20, 17, 3, 0, ws).shape == (4, 3, 340)
    d = torch.empty(3, 11, dtype=torch.float64, **meta)
    o = torch.empty(3, dtype=torch.float64, **meta)
    assert torch.ops.rt.trace(blob, 3, o, d, -1, 1, ws).shape == (3, 11)
    t = torch.empty(11, dtype=torch.float64, **meta)
    assert torch.ops.rt.shade_hits(blob, 3, 1, o, d, t, 3, 0, ws).dtype == torch.float32
    assert torch.ops.rt.intersect(blob[:8], o, d).shape == (11,)
    assert torch.ops.rt.quantize_u8(d).shape == (11, 3)
    assert torch.ops.rt.assemble_rows(torch.empty(2, 64, dtype=torch.uint8, **meta), 4, 4, 1, 2).shape == (4, 4, 3)
    # weighted shares (round 5): a run of parts per render, and the un-permute of unequal runs
    assert "int part_run=1" in str(torch.ops.rt.render_tile.default._schema)
    assert "int root_run=1, int run=1" in str(torch.ops.rt.assemble_rows.default._schema)
    for part, run in ((0, 1), (1, 2), (3, 2)):  # 17 rows in blocks of 2 over 5 parts, runs from `part`
        want = tiling.n_local_rows(17, 2, 5, part, run)
        got = torch.ops.rt.render_tile(blob, 3, 20, 17, 2, 5, part, 3, 2, ws, part_run=run)
        assert got.shape == (want, 20, 3), (part, run)
    with pytest.raises(RuntimeError, match="geometry"):
        torch.ops.rt.render_tile(blob, 3, 20, 17, 2, 5, 4, 3, 2, ws, part_run=2)  # past the interleave
    tiles = torch.empty(3, 64 * 9, dtype=torch.uint8, **meta)
    assert torch.ops.rt.assemble_rows(tiles, 8, 16, 2, 2, root_run=1, run=2).shape == (16, 8, 3)
    with pytest.raises(RuntimeError, match="run"):
        torch.ops.rt.assemble_rows(tiles, 8, 16, 2, 2, root_run=0, run=2)


def test_ops_refuse_a_variant_library():
    """RTX_HIP_LIB (an A/B variant of librtx_hip.so for HipRenderer) cannot be mixed with the ops,
    which link the in-tree library by $ORIGIN: importing the ops then raises ImportError."""
    code = ("import os, sys; sys.path.insert(0, os.getcwd())\n"
            "try:\n    import python_ray_tracer_amd.ops\nexcept ImportError as e:\n"
            "    print('refused:', e); sys.exit(0)\nsys.exit(3)\n")
    env = dict(os.environ, RTX_HIP_LIB=str(REPO / "python_ray_tracer_amd" / "variant_librtx_hip.so"))
    r = subprocess.run([sys.executable, "-c", code], cwd=str(REPO), env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "RTX_HIP_LIB" in r.stdout, r.stdout + r.stderr


def test_pack_image_texture():
    """An ImageTexture packs as RTX_TEX_IMAGE with its float64 texels (uint8 / 255.0, shape.py:65)
    appended once per distinct image; the material words hold the table offset, width, height."""
    from python_ray_tracer_amd.domain import Scene3D
    from python_ray_tracer_amd.infrastructure.hip import HipTexturedSphere, HipVector3D, ImageTexture

    sc = scenes.build_scene(scenes.random_spec(9, 2, 16, 9))  # 10 spheres: the culling tree too
    img = (np.arange(5 * 7 * 3).reshape(5, 7, 3) * 7 % 256).astype(np.uint8)
    a = HipTexturedSphere(HipVector3D(0, 0.5, 2), 0.7, img)
    b = HipTexturedSphere(HipVector3D(1, 0.5, 3), 0.4, img.copy())  # same content: one table
    blob = scene_pack.pack_scene(Scene3D(list(sc.shapes) + [a, b], sc.lights, sc.camera))
    S = 12
    mat = blob[L.HDR_WORDS + S * L.GEOM_WORDS:L.HDR_WORDS + S * (L.GEOM_WORDS + L.MAT_WORDS)].reshape(S, -1)
    assert mat[10, L.M_TEX] == L.TEX_IMAGE and mat[11, L.M_TEX] == L.TEX_IMAGE
    assert mat[10, L.M_TR] == mat[11, L.M_TR] and (mat[10, L.M_TG], mat[10, L.M_TB]) == (7, 5)
    off = int(mat[10, L.M_TR])
    assert off + 105 == blob.size and np.array_equal(blob[off:].reshape(5, 7, 3), img / 255.0)
    assert blob[L.H_NNODES] > 0  # the tree sits before the texels
    with pytest.raises(ValueError):
        ImageTexture(np.zeros((4, 4)))


def test_tame_flag():
    """RTX_H_TAME (the fast kernel's half-b sphere test): set when every sphere coordinate, radius
    and camera coordinate is below 2^60 in magnitude, cleared otherwise (and for non-finite ones)."""
    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import _lib as L
    from python_ray_tracer_amd.infrastructure.hip import scene_pack as P

    spec = scenes.readme_spec(8, 6)
    assert P.pack_scene(scenes.build_scene(spec))[L.H_TAME] == 1.0
    for key, val in (("center", [0.0, 0.0, 2.0 ** 61]), ("radius", 2.0 ** 60)):
        s2 = scenes.readme_spec(8, 6)
        s2["spheres"][0][key] = val
        assert P.pack_scene(scenes.build_scene(s2))[L.H_TAME] == 0.0, key
    s3 = scenes.readme_spec(8, 6)
    s3["camera"]["position"] = [0.0, -3e18, 0.0]
    assert P.pack_scene(scenes.build_scene(s3))[L.H_TAME] == 0.0


def test_pack_override_material():
    """NumpyShader.create on another shape's shader: the blob is the scene's own plus one material
    record (RTX_H_MAT0 points at it) packed from that shader, whose image texels (if any) follow it;
    everything else is unchanged (the reflections see the scene as it is, shader.py:152)."""
    from python_ray_tracer_amd.infrastructure.hip import HipShader, ImageTexture

    sc = scenes.build_scene(scenes.random_spec(16, 0, 32, 18))
    base = scene_pack.pack_scene(sc)
    assert base[L.H_MAT0] == 0
    shape, other = sc.shapes[9], sc.shapes[3].shader
    blob = scene_pack.pack_override(sc, shape, other)
    off = int(blob[L.H_MAT0])
    assert off == base.size and blob.size == base.size + L.MAT_WORDS
    assert np.array_equal(np.delete(blob[:base.size], L.H_MAT0), np.delete(base, L.H_MAT0))
    S = 17
    own3 = base[L.HDR_WORDS + S * L.GEOM_WORDS + 3 * L.MAT_WORDS:][:L.MAT_WORDS]
    assert np.array_equal(blob[off:off + L.MAT_WORDS], own3)  # shape 3's material record, verbatim
    img = (np.arange(4 * 6 * 3).reshape(4, 6, 3) * 11 % 256).astype(np.uint8)
    tex = HipShader(0.0, 0.2, 0.5, 0.0, 1.0, ImageTexture(img))
    blob = scene_pack.pack_override(sc, shape, tex)
    off = int(blob[L.H_MAT0])
    assert blob[off + L.M_TEX] == L.TEX_IMAGE and int(blob[off + L.M_TR]) == off + L.MAT_WORDS
    assert np.array_equal(blob[off + L.MAT_WORDS:].reshape(4, 6, 3), img / 255.0)


@pytest.mark.parametrize("n_spheres,light", [(64, None), (16, [1.5, 2.0, 6.0]), (40, [0.3, 0.6, 8.0]), (8, None),
                                             (9, [-1.0, 0.2, 3.0]), (12, [0.0, 0.1, 30.0]),
                                             (24, [0.5, 0.0, 6.0]), (16, [0.0, -0.4, 3.0])])
def test_shadow_grid_masks_are_conservative(n_spheres, light):
    """scene_pack's shadow grid (RTX_H_SHGRID): for hit points sampled on every sphere's surface and
    on the ground (inside and far outside the grid), any sphere the reference's shadow test
    (shader.py:126-128: oracle.intersect from the nudged point along L_dir) reports as hit must be in
    the mask the kernel would pick (rtx_kernels.hip grid_mask): the voxel's when the nudged point lies
    in the grid, else the huge spheres' when the ray's line misses the small spheres' ball."""
    spec = scenes.random_spec(n_spheres, 7, 64, 36)
    if light is not None:
        spec["lights"][0]["position"] = light
    sc = O.scene_from_spec(spec)
    blob = scene_pack.pack_scene(scenes.build_scene(spec))
    off = int(blob[L.H_SHGRID])
    assert off > 0
    g = blob[off:off + L.SHGRID_WORDS]
    nx, ny, nz = (int(v) for v in g[6:9])
    nvox = nx * ny * nz
    masks = blob[off + L.SHGRID_WORDS: off + L.SHGRID_WORDS + 2 * (nvox + 1)].view(np.uint64).reshape(-1, 2)
    rng = np.random.default_rng(11)
    lx0, ly0, lz0 = sc.light_pos
    checked = {"voxel": 0, "outside": 0}
    for si, sp in enumerate(sc.spheres):
        m = 6000 if sp.radius > 100 else 400
        if sp.radius > 100:  # the ground: under the grid and up to 3x its extent around it
            ex, ez = nx / g[3], nz / g[5]
            x = rng.uniform(g[0] - ex, g[0] + 2 * ex, m)
            z = rng.uniform(g[2] - ez, g[2] + 2 * ez, m)
            y = sp.cy + np.sqrt(sp.radius ** 2 - (x - sp.cx) ** 2 - (z - sp.cz) ** 2)
            u = np.stack([(x - sp.cx) / sp.radius, (y - sp.cy) / sp.radius, (z - sp.cz) / sp.radius])
        else:
            u = rng.normal(size=(3, m))
            u /= np.sqrt((u ** 2).sum(axis=0))
        px, py, pz = sp.cx + sp.radius * u[0], sp.cy + sp.radius * u[1], sp.cz + sp.radius * u[2]
        inv_r = 1.0 / sp.radius
        nxv, nyv, nzv = (px - sp.cx) * inv_r, (py - sp.cy) * inv_r, (pz - sp.cz) * inv_r
        lx, ly, lz = O._norm(lx0 - px, ly0 - py, lz0 - pz)
        qx, qy, qz = px + nxv * 0.0001, py + nyv * 0.0001, pz + nzv * 0.0001
        fx, fy, fz = (qx - g[0]) * g[3], (qy - g[1]) * g[4], (qz - g[2]) * g[5]
        n2 = (nxv * nxv + nyv * nyv) + nzv * nzv
        inside = (fx >= 0) & (fx < nx) & (fy >= 0) & (fy < ny) & (fz >= 0) & (fz < nz) & (n2 <= 4.0)
        key = np.where(inside, (np.clip(fz, 0, nz - 1).astype(np.int64) * ny + np.clip(fy, 0, ny - 1).astype(np.int64))
                       * nx + np.clip(fx, 0, nx - 1).astype(np.int64), nvox)
        wx, wy, wz = g[9] - qx, g[10] - qy, g[11] - qz
        ww = (wx * wx + wy * wy) + wz * wz
        hh = (wx * lx + wy * ly) + wz * lz
        qq = (qx * qx + qy * qy) + qz * qz
        R = (g[12] + 5e-7 * (qq + 1.0)) + 3e-8 * (ww + 1.0)
        usable = inside | (ww - hh * hh > R * R)
        for j, other in enumerate(sc.spheres):
            if j == si:
                continue  # the own shape never shadows (t_self < t_self is false)
            t = O.intersect(other, qx, qy, qz, lx, ly, lz)
            hit = usable & (t < O.FARAWAY)
            if not hit.any():
                continue
            bits = masks[key[hit], j >> 6] >> np.uint64(j & 63) & np.uint64(1)
            assert bits.all(), (si, j, int((bits == 0).sum()))
            checked["voxel"] += int((hit & inside).sum())
            checked["outside"] += int((hit & ~inside).sum())
    assert checked["voxel"] > 10, checked


def _beam_candidates(G, Oc, A, r2, omc, drop_rho=False):
    """Numpy restatement of rtx_kernels.hip wave_beam for one wave: G = [S, 4] (centre, radius),
    Oc / A the first active lane's origin / direction, r2 / omc the active lanes' |O - Oc|^2 and
    1 - D.A. Returns the candidate flags, or None where the kernel falls back to the culling tree."""
    def p2above(x, lo, hi):
        e = np.frexp(x)[1]
        e = np.where(x < 2.0 ** (lo - 1), lo, np.maximum(e, lo))
        return np.where(~(x < 2.0 ** hi), hi + 1, e)

    er, ea = int(p2above(r2, -60, 12).max()), int(p2above(omc, -60, -1).max())
    if er > 12 or ea > -1:
        return None
    # the kernel's bounds (round 6: the test squared, no square root of |W|^2 - R^2; sqrt_cull is
    # within ~1e-15 of the square root, the callers' 1 + 1e-11 keeps every bound on the safe side)
    rho2 = 0.0 if drop_rho else 2.0 ** er
    rho = np.sqrt(rho2) * (1 + 1e-11)
    ct = 1 - 2.0 ** ea
    ct2, st = (ct * ct) * (1 - 1e-12), np.sqrt(2.0 ** (ea + 1)) * (1 + 1e-11)
    lmk = ((2 * rho2 + 2 * (Oc @ Oc)) + 2 * rho2) + 1.0
    Wv = G[:, :3] - Oc
    ww = (Wv ** 2).sum(1)
    rr, CC = G[:, 3] ** 2, (G[:, :3] ** 2).sum(1)
    lm = 4e-7 * ((((2 * ww + 2 * CC) + 3 * rr) + lmk) * (1 + 1e-12))
    R = ((np.sqrt(rr) * (1 + 1e-11) + lm) + rho) * (1 + 1e-12)
    R2 = R * R
    t1 = (Wv @ A + st * R) + 1e-9 * ((ww + R2) + 2.0)
    drop = (ww > R2 * (1 + 1e-12)) & ((t1 < 0) | (t1 * t1 < ((ww - R2) - 1e-15 * (ww + R2)) * ct2))
    return ~drop


@pytest.mark.parametrize("seed", [0, 3])
def test_wave_beam_is_conservative(seed):
    """The reflected-ray beam cull (rtx_kernels.hip wave_beam, levels >= 1 of scenes of 32 spheres and
    more): for every 8x8 wave tile and random subsets of its live lanes (the lanes still bouncing), any
    sphere that the reference's intersect (shape.py:28-51, oracle) reports a hit for on a live lane's
    reflected ray must be a candidate. Mutation check: without the origin ball's radius rho some
    wave loses a hit sphere."""
    spec = scenes.random_spec(64, seed, 160, 96)
    sc = O.scene_from_spec(spec)
    W, H = 160, 96
    G = np.array([[sp.cx, sp.cy, sp.cz, sp.radius] for sp in sc.spheres])
    dx, dy, dz = O.ray_directions(sc.cam, W, H)
    ox, oy, oz = (np.full(W * H, c) for c in sc.cam)
    alive = np.ones(W * H, bool)
    idx = np.arange(W * H)
    tile = (idx // W // 8) * (W // 8) + (idx % W) // 8
    rng = np.random.default_rng(seed)
    stats = {"waves": 0, "hits": 0, "mutant_misses": 0}
    for level in range(4):
        dist = np.stack([np.broadcast_to(O.intersect(sp, ox, oy, oz, dx, dy, dz), (W * H,)) for sp in sc.spheres])
        if level >= 1:
            for t in np.unique(tile[alive]):
                lanes = np.nonzero((tile == t) & alive)[0]
                for sub in (lanes, lanes[rng.random(lanes.size) < 0.5]):
                    if sub.size == 0:
                        continue
                    f = sub[0]
                    Oc, A = np.array([ox[f], oy[f], oz[f]]), np.array([dx[f], dy[f], dz[f]])
                    r2 = (ox[sub] - Oc[0]) ** 2 + (oy[sub] - Oc[1]) ** 2 + (oz[sub] - Oc[2]) ** 2
                    omc = 1.0 - (dx[sub] * A[0] + dy[sub] * A[1] + dz[sub] * A[2])
                    cand = _beam_candidates(G, Oc, A, r2, omc)
                    if cand is None:
                        continue
                    stats["waves"] += 1
                    hit = (dist[:, sub] < O.FARAWAY).any(axis=1)
                    stats["hits"] += int(hit.sum())
                    assert not (hit & ~cand).any(), (level, t, np.nonzero(hit & ~cand)[0])
                    mutant = _beam_candidates(G, Oc, A, r2, omc, drop_rho=True)
                    stats["mutant_misses"] += int((hit & ~mutant).sum())
        near = dist.min(0)
        hit_s = np.where(near < O.FARAWAY, dist.argmin(0), -1)
        nxt = [a.copy() for a in (ox, oy, oz, dx, dy, dz)]
        nalive = np.zeros_like(alive)
        for si, sp in enumerate(sc.spheres):
            ii = np.nonzero(alive & (hit_s == si))[0]
            if ii.size == 0:
                continue
            _, _, lit, _, q, r = O._shade(sc, si, sp, ox[ii], oy[ii], oz[ii], dx[ii], dy[ii], dz[ii], near[ii])
            j = ii[lit & (sp.specular_gain != 0)]
            for a, v in zip(nxt, (*q, *r)):
                a[j] = v[lit & (sp.specular_gain != 0)]
            nalive[j] = True
        ox, oy, oz, dx, dy, dz = nxt
        alive = nalive
    assert stats["waves"] > 200 and stats["hits"] > 200, stats
    assert stats["mutant_misses"] > 0, stats


def test_pack_sin_range_flag():
    """RTX_H_SINRED: set when every material's thin-film phase (at most 10 pi |thickness|,
    shader.py:204-208) lies in the kernel sine's reduction range; a thickness beyond it (also on
    Shader.create's override material) clears it, and the kernel then checks every wave."""
    from python_ray_tracer_amd.infrastructure.hip import HipShader

    spec = scenes.random_spec(5, 1, 16, 9)
    assert scene_pack.pack_scene(scenes.build_scene(spec))[L.H_SINRED] == 1.0
    sc = scenes.build_scene(spec)
    far = HipShader(0.5, 0.5, 0.5, 0.1, 1.0, sc.shapes[0].shader.diffuse_color)
    far.thin_film_thickness = 1e5
    assert scene_pack.pack_override(sc, sc.shapes[1], far)[L.H_SINRED] == 0.0
    near = HipShader(0.5, 0.5, 0.5, 0.1, 1.0, far.diffuse_color)
    near.thin_film_thickness = 3e4
    assert scene_pack.pack_override(sc, sc.shapes[1], near)[L.H_SINRED] == 1.0
    sc.shapes[2].shader.thin_film_thickness = -1e5
    assert scene_pack.pack_scene(sc)[L.H_SINRED] == 0.0


@pytest.mark.parametrize("layout", sorted(HUGE_LAYOUTS))
def test_pack_huge_tail(layout):
    """RTX_H_NBEAM: the first index of the huge spheres that end the scene (every later sphere huge,
    so the kernel's tile frustums and reflected-ray beams take them without a test); 0 when the last
    sphere is small."""
    spec = huge_tail_spec(layout, 32, 18)
    blob = scene_pack.pack_scene(scenes.build_scene(spec))
    nb, S = int(blob[L.H_NBEAM]), len(spec["spheres"])
    assert nb == HUGE_LAYOUTS[layout][-1]
    radii = [sp["radius"] for sp in spec["spheres"]]
    if nb:
        assert all(r > scene_pack.HUGE_RADIUS for r in radii[nb:]) and radii[nb - 1] <= scene_pack.HUGE_RADIUS
    else:
        assert radii[-1] <= scene_pack.HUGE_RADIUS
    assert 0 <= nb < S


@pytest.mark.parametrize("case", ["c4", "c3", "cam_ahead", "cam_behind", "inside", "near_plane"])
def test_plane_boxes_are_conservative(case):
    """RTX_H_SBOX (scene_pack.sphere_plane_boxes): every camera ray the reference's intersect
    (shape.py:28-51) reports a hit for passes through an image-plane point inside that sphere's box,
    for every pixel of a small frame and for dense plane points around each bounded box; shrinking
    the boxes by 0.5% of their size loses hits (the test has teeth)."""
    spec = scenes.random_spec(64 if case == "c4" else 16, 3, 160, 90)
    cam = {"c4": None, "c3": None, "cam_ahead": [0.4, 0.8, -0.7], "cam_behind": [0.3, 0.9, 18.0],
           "inside": None, "near_plane": [0.0, 0.6, -0.05]}[case]
    if cam is not None:
        spec["camera"]["position"] = cam
    if case == "inside":  # the camera inside a sphere: that sphere's box is unbounded
        spec["spheres"][0]["center"] = [float(v) + 0.1 for v in spec["camera"]["position"]]
        spec["spheres"][0]["radius"] = 0.8
    sc = O.scene_from_spec(spec)
    blob = scene_pack.pack_scene(scenes.build_scene(spec))
    off = int(blob[L.H_SBOX])
    assert off > 0
    S = len(sc.spheres)
    box = blob[off:off + 4 * S].reshape(S, 4)
    ox, oy, oz = sc.cam
    W, H = sc.width, sc.height
    aspect = W / H
    px = np.tile(np.linspace(-1, 1, W), H)
    py = np.repeat(np.linspace(1 / aspect + 0.25, -1 / aspect + 0.25, H), W)
    rng = np.random.default_rng(5)
    for b in box:  # dense points around each bounded box
        if np.all(np.isfinite(b)):
            cx, cy, ex, ey = (b[0] + b[1]) / 2, (b[2] + b[3]) / 2, (b[1] - b[0]) * 0.6, (b[3] - b[2]) * 0.6
            px = np.concatenate([px, rng.uniform(cx - ex, cx + ex, 3000)])
            py = np.concatenate([py, rng.uniform(cy - ey, cy + ey, 3000)])
    dx, dy, dz = O._norm(px - ox, py - oy, 0 - oz)
    hits = lost = 0
    for j, sp in enumerate(sc.spheres):
        hit = O.intersect(sp, ox, oy, oz, dx, dy, dz) < O.FARAWAY
        lo_x, hi_x, lo_y, hi_y = box[j]
        inside = (px >= lo_x) & (px <= hi_x) & (py >= lo_y) & (py <= hi_y)
        assert not (hit & ~inside).any(), (case, j, box[j], int((hit & ~inside).sum()))
        hits += int(hit.sum())
        if np.all(np.isfinite(box[j])):
            sx, sy = (hi_x - lo_x) * 0.005, (hi_y - lo_y) * 0.005
            shrunk = (px >= lo_x + sx) & (px <= hi_x - sx) & (py >= lo_y + sy) & (py <= hi_y - sy)
            lost += int((hit & ~shrunk).sum())
    assert hits > 100, hits
    if case != "inside":
        assert lost > 0, case
    if case == "inside":
        assert np.all(np.isinf(box[0]))
