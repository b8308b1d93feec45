"""GPU parity at the BASELINE configs' own sizes.

C2 (1920x1080, B=3) is in test_gpu_parity.py. The others are rendered here at full size on the GPU
and compared with the CPU oracle (max-abs <= 1e-12 on float64 colour, identical uint8, per-level
ray/hit counters equal). That exercises what reduced sizes do not: the culling tree's margins
over the whole frame, the frame-size-scaled resume-record capacities, the persistent wave-tile
fetch of >= 32-sphere scenes over 518,400 wave tiles (C4), and the 32-frame batched launch (C5).

Where the oracle would take minutes (C4 is 33 M pixels and 65 spheres), the GPU renders the whole
frame and the oracle renders a few interleaved row tiles of it (``render_rows``): reference pixels
are independent (every array op is elementwise per ray, base.py:91-141), so those rows of the
oracle's full frame are exactly ``render_rows``.
"""

import numpy as np
import pytest
import torch

from oracle import numpy_oracle as O
from python_ray_tracer_amd import scenes, tiling

pytestmark = pytest.mark.gpu

ATOL = 1e-12


@pytest.fixture(scope="module")
def hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from python_ray_tracer_amd.infrastructure import hip as H

    return H


def _rows_of(frame: torch.Tensor, rows, W: int) -> np.ndarray:
    """[3, H*W] device frame -> [3, len(rows)*W] host array of the given rows."""
    idx = torch.as_tensor(np.asarray(rows), device=frame.device)
    return frame.reshape(3, -1, W)[:, idx].reshape(3, -1).cpu().numpy()


def _check(got, want, W, H, label):
    err = float(np.abs(got - want).max())
    assert err <= ATOL, (label, err)
    assert np.array_equal(O.to_uint8(got, W, H), O.to_uint8(want, W, H)), label


def test_c1_readme_960x540_full_frame(hip):
    """configs[0]: the README scene at 960x540, B=3, whole frame, counters equal."""
    spec, B = scenes.CONFIGS["C1"]()
    r = hip.HipRenderer(max_bounces=B, collect_stats=True)
    scene = scenes.build_scene(spec)
    got = r.raytrace_scene(scene.camera.position, r.get_ray_directions(scene.camera), scene).data.cpu().numpy()
    st = O.TraceStats()
    want = O.render(O.scene_from_spec(spec), B, stats=st)
    _check(got, want, 960, 540, "C1")
    s = r.stats()
    assert s["rays"] == st.rays and s["hits"] == st.hits
    assert s["pixels"] == 960 * 540


def test_c3_4k_16_spheres_full_frame(hip):
    """configs[2]: 3840x2160, 16 spheres + ground, B=4, the whole frame against the oracle. The
    whole frame's launch (8.3 M pixels) runs the one-tile kernel built for 6 waves/SIMD
    (kFwdWavesLarge, launches of 4 M pixels and more); three interleaved row tiles of 2.8 M pixels
    each run the 5-wave build, and give the same rows bit for bit."""
    spec, B = scenes.CONFIGS["C3"]()
    r = hip.HipRenderer(max_bounces=B, collect_stats=True)
    scene = scenes.build_scene(spec)
    frame = r.render(scene).data
    got = frame.cpu().numpy()
    st = O.TraceStats()
    want = O.render(O.scene_from_spec(spec), B, stats=st)
    _check(got, want, 3840, 2160, "C3")
    s = r.stats()
    assert s["rays"] == st.rays and s["hits"] == st.hits
    r5 = hip.HipRenderer(max_bounces=B)
    for part in range(3):
        rows = tiling.tile_rows(2160, 8, 3, part)
        assert 3840 * len(rows) < 4 << 20
        assert np.array_equal(r5.render_tile(scene, 8, 3, part).cpu().numpy(), _rows_of(frame, rows, 3840)), part


# row tiles of the 64-way interleaved split of C4 (8-row blocks) checked against the oracle
C4_PARTS = (0, 29, 63)


@pytest.fixture(scope="module")
def c4(hip):
    spec, B = scenes.CONFIGS["C4"]()
    return spec, B, scenes.build_scene(spec), O.scene_from_spec(spec)


def test_c4_8k_64_spheres_full_frame_rows(hip, c4):
    """configs[3] on one GPU: the whole 7680x4320 frame (65 spheres, B=5: the persistent
    wave-tile launch and the culling tree), three interleaved row tiles against the oracle; the
    8-way row tile a rank renders equals the same rows of the whole frame; the counters of one
    64-way tile equal the oracle's."""
    spec, B, scene, osc = c4
    W, H = 7680, 4320
    r = hip.HipRenderer(max_bounces=B)
    frame = r.render(scene).data
    for part in C4_PARTS:
        rows = tiling.tile_rows(H, 8, 64, part)
        want = O.render_rows(osc, rows, B)
        _check(_rows_of(frame, rows, W), want, W, len(rows), f"C4 part {part}")
    # the tile rank 5 of 8 renders = rows 5 (mod 8 blocks) of the full frame, bit for bit
    tile = r.render_tile(scene, 8, 8, 5)
    rows8 = tiling.tile_rows(H, 8, 8, 5)
    assert np.array_equal(tile.cpu().numpy(), _rows_of(frame, rows8, W))
    rs = hip.HipRenderer(max_bounces=B, collect_stats=True)
    rs.render_tile(scene, 8, 64, 29)
    st = O.TraceStats()
    O.render_rows(osc, tiling.tile_rows(H, 8, 64, 29), B, stats=st)
    s = rs.stats()
    assert s["rays"] == st.rays and s["hits"] == st.hits


def test_c4_unbounded_full_frame_rows(hip, c4):
    """C4 with the reference's unbounded recursion at full size (the DEEP pipeline: a first pass
    that defers a chain still alive at level 30 with a 10-word resume record, one continuation pass
    to level 60, the general kernel beyond; capacities scaled with the 33 M-pixel frame); sampled
    rows vs the oracle. Whether C4 has chains past level 30 depends on the scene: the records and
    both resumes are exercised deterministically by test_gpu_parity.py::
    test_deep_chains_resume_past_levels_30_and_60 (every chain of a trapped-ray scene passes
    levels 31 and 61), and this test also checks whether any chain of C4 was deferred at all."""
    spec, _, scene, osc = c4
    W, H = 7680, 4320
    r = hip.HipRenderer()  # max_bounces=None
    frame = r.render(scene).data
    for part in (0, 63):
        rows = tiling.tile_rows(H, 8, 64, part)
        want = O.render_rows(osc, rows, None)
        _check(_rows_of(frame, rows, W), want, W, len(rows), f"C4 unbounded part {part}")
    # the counting render: per-level rays match the capped render's below its cap, and the deepest
    # level reached is printed (a chain alive at level 30 went through a resume record)
    rs = hip.HipRenderer(collect_stats=True)
    rs.render(scene)
    st = rs.stats()
    print(f"C4 unbounded: deepest level {len(st['rays']) - 1}, rays past level 30: {sum(st['rays'][31:])}, "
          f"deferred to the general kernel: {st['deferred']}")
    assert len(st["rays"]) > 6  # chains beyond the capped kernel's levels exist


def test_c5_orbit_32_frame_batch(hip):
    """configs[4]: one rank's 32 frames of the 256-frame 1080p orbit in ONE launch
    (rtx_render_frames), frames {0, 37, 128, 255} against the oracle; every frame of the batch
    equals its single-frame render."""
    spec, B = scenes.CONFIGS["C5"]()
    ks = sorted(set(range(0, 256, 9)) | {0, 37, 128, 255})[:32]
    assert len(ks) == 32 and {0, 37, 128, 255} <= set(ks)
    frames = [scenes.build_scene(scenes.with_camera(spec, scenes.orbit_position(k, 256))) for k in ks]
    r = hip.HipRenderer(max_bounces=B)
    batch = r.render_batch(frames)
    assert batch.shape == (32, 3, 1920 * 1080)
    for k in (0, 37, 128, 255):
        f = ks.index(k)
        want = O.render(O.scene_from_spec(scenes.with_camera(spec, scenes.orbit_position(k, 256))), B)
        _check(batch[f].cpu().numpy(), want, 1920, 1080, f"C5 frame {k}")
    for f in range(0, 32, 5):
        assert torch.equal(batch[f], r.render_tile(frames[f])), f
