"""Pin the CPU oracle to the reference: fixtures produced by running the reference itself
(tests/golden/make_golden.py) and the reference's committed render.png."""

import hashlib
import json

import numpy as np
import pytest

from oracle import numpy_oracle as O
from python_ray_tracer_amd import scenes
from tests.conftest import GOLDEN, golden_png, same_platform


def test_cases_bit_exact(golden_meta, golden_renders):
    exact = same_platform(golden_meta)
    for name, case in golden_meta["cases"].items():
        sc = O.scene_from_spec(case["spec"])
        st = O.TraceStats()
        out = O.render(sc, case["max_bounces"], trace_all=True, stats=st)
        ref = golden_renders[name]
        if exact:
            assert np.array_equal(out, ref), name
        else:  # other CPU: NumPy's SIMD sin/pow may differ by an ulp
            np.testing.assert_allclose(out, ref, rtol=0, atol=1e-12, err_msg=name)
        # trace_all reproduces the reference's own per-level ray / shaded-hit counts
        assert st.rays == case["rays"], name
        assert st.hits == case["hits"], name


def test_skipping_zero_weight_rays_changes_nothing(golden_meta, golden_renders):
    for name in ("main_160x90_B3", "readme_160x90_Binf", "rand16_128x72_B4", "ties_64x36_B2"):
        case = golden_meta["cases"][name]
        a = O.render(O.scene_from_spec(case["spec"]), case["max_bounces"])
        b = O.render(O.scene_from_spec(case["spec"]), case["max_bounces"], trace_all=True)
        assert np.array_equal(a, b), name


def test_ties_are_exercised(golden_meta):
    case = golden_meta["cases"]["ties_64x36_B2"]
    st = O.TraceStats()
    O.render(O.scene_from_spec(case["spec"]), 2, stats=st)
    assert st.ties > 100


def test_render_png_byte_exact():
    """main.py (unbounded bounces) reproduces the reference's committed render.png."""
    png = golden_png("render_main_960x540.png")
    out = O.render(O.scene_from_spec(scenes.main_spec(960, 540)), None)
    assert np.array_equal(O.to_uint8(out, 960, 540), png)


@pytest.mark.parametrize("tag", ["main", "readme"])
def test_1080p_against_reference(golden_meta, tag):
    m = golden_meta[f"ref_1080p_B3_{tag}"]
    st = O.TraceStats()
    out = O.render(O.scene_from_spec(m["spec"]), 3, trace_all=True, stats=st)
    assert st.rays == m["rays"] and st.hits == m["hits"]
    assert np.array_equal(O.to_uint8(out, 1920, 1080), golden_png(f"ref_1080p_B3_{tag}.png"))
    if same_platform(golden_meta):
        assert hashlib.sha256(np.ascontiguousarray(out).tobytes()).hexdigest() == m["sha256_f64"]
    else:
        assert abs(float(out.sum()) - m["sum"]) <= 1e-9 * abs(m["sum"])


def test_intersect_known_answers():
    kat = json.loads((GOLDEN / "intersect_kat.json").read_text())
    for k in kat:
        sp = O.OSphere(*k["center"], k["radius"], 0, 0, 0, 0, 0, False, (1, 1, 1))
        d = [np.array([v]) for v in k["dir"]]
        t = O.intersect(sp, *[float(v) for v in k["origin"]], *d)[0]
        assert t == k["t"], k["label"]
    labels = {k["label"]: k["t"] for k in kat}
    assert labels["hit front (test_objects.py:6-11)"] == 2.0
    assert labels["miss (test_objects.py:14-19)"] == O.FARAWAY
    assert labels["tangent: disc == 0 is a miss"] == O.FARAWAY
    assert labels["origin inside: far root"] == 1.0
    assert labels["sphere behind the origin"] == O.FARAWAY


def test_norm_known_answer():
    want = json.loads((GOLDEN / "vector_kat.json").read_text())["norm_3_4_0"]
    got = O._norm(np.float64(3), np.float64(4), np.float64(0))
    assert [float(v) for v in got] == want == [0.6000000000000001, 0.8, 0.0]


def test_ray_directions_match_numpy_linspace():
    for W, H in ((1, 1), (7, 5), (160, 90), (1920, 1080)):
        dx, dy, dz = O.ray_directions((0, 0.2, -2), W, H)
        assert dx.shape == (W * H,)
        xs = np.tile(np.linspace(-1, 1, W), H)
        assert np.all(np.sign(dx) == np.sign(xs))  # sanity: row-major, x from -1 to 1


def test_flop_model():
    assert O.flop_model(10, 4, 20, 5) == 150 + 20 * 4 * 25 + 1000


def test_oracle_create_matches_reference_fixtures():
    """O.create == the reference NumpyShader.create called directly (shader.py:63-112), on rays
    that hit the shape whether or not it is their nearest, capped and unbounded
    (tests/golden/make_golden_create.py)."""
    import json

    z = np.load(GOLDEN / "create_kat.npz")
    meta = json.loads((GOLDEN / "create_kat.json").read_text())
    for name, c in meta["cases"].items():
        sc = O.scene_from_spec(c["spec"])
        other = c.get("shader_of", c["shape"])
        mat = sc.spheres[other] if other != c["shape"] else None  # create on another shape's shader
        got = np.stack(O.create(sc, c["shape"], tuple(c["origin"]), tuple(z[name + "_dirs"]), z[name + "_t"],
                                c["max_bounces"], material=mat))
        assert np.abs(got - z[name + "_rgb"]).max() <= 1e-12, name


def test_oracle_render_rows_equals_full_frame_rows():
    from python_ray_tracer_amd import tiling

    spec = scenes.random_spec(16, 1, 64, 37)
    sc = O.scene_from_spec(spec)
    full = O.render(sc, 4).reshape(3, 37, 64)
    for P, p in ((3, 1), (5, 4)):
        rows = tiling.tile_rows(37, 4, P, p)
        assert np.array_equal(O.render_rows(sc, rows, 4), full[:, rows].reshape(3, -1))


def test_oracle_image_texels_match_reference_textured_sphere():
    """O.image_texels == the reference NumpyTexturedSphere.diffusecolor (shape.py:66-79) evaluated
    on single points (tests/golden/make_golden_texture.py): random points, poles, the u seam."""
    import json

    k = json.loads((GOLDEN / "texture_kat.json").read_text())
    sp = O.OSphere(*k["center"], k["radius"], 0, 0, 0, 0, 1, False, (1, 1, 1),
                   image=np.asarray(k["image"], dtype=np.uint8) / 255.0)
    P = np.asarray(k["points"])
    got = np.stack(O.image_texels(sp, P[:, 0], P[:, 1], P[:, 2]), 1)
    assert np.array_equal(got, np.asarray(k["rgb"]))
