"""Generate the golden fixtures in this directory by running the REFERENCE renderer.

Run in the build container only (it needs ``/root/reference``, which never travels to the GPU box):

    python tests/golden/make_golden.py

What it writes (all small, committed):

* ``renders.npz``      float64 RGB outputs of the reference ``NumpyRenderer`` (``base.py:91-141``)
                       for several scenes / sizes / bounce caps, plus per-level ray and hit counts.
* ``scenes.json``      the scene specs (``python_ray_tracer_amd/scenes.py`` format) and metadata
                       (numpy version, CPU flags — NumPy's SIMD ``sin``/``pow`` are only ulp-exact on
                       the same dispatch target).
* ``intersect_kat.json`` known-answer ``NumpySphere.intersect`` cases (the intent of
                       the reference's dead ``tests/test_objects.py:6-19``).
* ``render_main_960x540.png`` a copy of the reference's committed ``render.png`` (the output of
                       ``main.py`` with unbounded bounces) — a data file of the reference.
* ``ref_1080p_B3_*.png`` the reference's own 1920x1080, 3-bounce uint8 output for the main and README
                       scenes, and the SHA-256 of its float64 output (``scenes.json``).

The reference requires Python >= 3.12 only for ``typing.Self``; a one-line shim provides it.
The bounce cap, absent from the reference, is a subclass that returns black past depth B — every
recursive call goes through ``self.raytrace_scene`` (``shader.py:152``), so the override sees all
levels.
"""

from __future__ import annotations

import hashlib
import json
import platform
import shutil
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path("/root/reference")

sys.path.insert(0, str(REPO))
from python_ray_tracer_amd import scenes as S  # noqa: E402  (spec builders only)


def _import_reference():
    import typing

    import typing_extensions

    typing.Self = typing_extensions.Self
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF))
    from ray_tracer.domain import Camera, DomeLight, PointLight, Scene3D
    from ray_tracer.infrastructure.numpy.base import NumpyRenderer, NumpyRGBColor, NumpyVector3D
    from ray_tracer.infrastructure.numpy.shader import NumpyShader, Texture, TextureChecker
    from ray_tracer.infrastructure.numpy.shape import NumpySphere

    return dict(Camera=Camera, DomeLight=DomeLight, PointLight=PointLight, Scene3D=Scene3D,
                NumpyRenderer=NumpyRenderer, NumpyRGBColor=NumpyRGBColor, NumpyVector3D=NumpyVector3D,
                NumpyShader=NumpyShader, Texture=Texture, TextureChecker=TextureChecker, NumpySphere=NumpySphere)


R = _import_reference()


def ref_scene(spec):
    V, C = R["NumpyVector3D"], R["NumpyRGBColor"]
    shapes = []
    for s in spec["spheres"]:
        sh = s["shader"]
        tex = R["TextureChecker"]() if sh["texture"]["kind"] == "checker" else R["Texture"](C(*sh["texture"]["color"]))
        shader = R["NumpyShader"](sh["reflection_gain"], sh["specular_gain"], sh["specular_roughness"],
                                  sh["iridescence_gain"], sh["diffuse_gain"], tex)
        shapes.append(R["NumpySphere"](V(*s["center"]), s["radius"], shader))
    lights = []
    for li in spec["lights"]:
        if li["kind"] == "point":
            lights.append(R["PointLight"](V(*li["position"])))
        else:
            lights.append(R["DomeLight"](li["intensity"], C(*li["color"])))
    cam = spec["camera"]
    return R["Scene3D"](shapes, lights, R["Camera"](V(*cam["position"]), cam["width"], cam["height"]))


class CappedRenderer(R["NumpyRenderer"]):
    """Reference NumpyRenderer with a bounce cap and per-level counters."""

    def __init__(self, max_bounces):
        self.max_bounces = max_bounces
        self.depth = 0
        self.rays = {}
        self.hits = {}

    def raytrace_scene(self, ray_origin, normalized_ray_direction, scene):
        if self.max_bounces is not None and self.depth > self.max_bounces:
            return R["NumpyRGBColor"](0, 0, 0)
        lvl = self.depth
        n = np.size(normalized_ray_direction.x)
        self.rays[lvl] = self.rays.get(lvl, 0) + int(n)
        self.depth += 1
        try:
            out = super().raytrace_scene(ray_origin, normalized_ray_direction, scene)
        finally:
            self.depth -= 1
        return out


class _CountingShaderHook:
    """Counts shaded hits per level by wrapping each shader's ``create``."""

    def __init__(self, scene, renderer):
        for shape in scene.shapes:
            sh = shape.shader
            if getattr(sh, "_wrapped", False):
                continue
            orig = sh.create

            def create(shape_, scene_, O, D, t, rt, _orig=orig):
                lvl = rt.depth - 1
                rt.hits[lvl] = rt.hits.get(lvl, 0) + int(np.size(t))
                return _orig(shape_, scene_, O, D, t, rt)

            sh.create = create
            sh._wrapped = True


def ref_render(spec, max_bounces):
    scene = ref_scene(spec)
    rend = CappedRenderer(max_bounces)
    _CountingShaderHook(scene, rend)
    dirs = rend.get_ray_directions(scene.camera)
    col = rend.raytrace_scene(scene.camera.position, dirs, scene)
    n = spec["camera"]["width"] * spec["camera"]["height"]
    out = np.stack([np.broadcast_to(np.asarray(c, dtype=np.float64), (n,)) for c in col.components()])
    levels = max(rend.rays) + 1
    rays = [rend.rays.get(i, 0) for i in range(levels)]
    hits = [rend.hits.get(i, 0) for i in range(levels)]
    return out, rays, hits, scene, rend, col


def tie_spec():
    """Two coincident spheres (identical centre and radius): every ray that hits one ties with the
    other, so both are shaded and summed (base.py:102-119). Plus a mirror sphere to reflect them."""
    spec = S.readme_spec(64, 36)
    dup = json.loads(json.dumps(spec["spheres"][1]))
    dup["shader"]["texture"] = {"kind": "const", "color": [0.1, 0.9, 0.2]}
    dup["shader"]["specular_gain"] = 0.6
    spec["spheres"].insert(2, dup)
    return spec


def inside_spec():
    """Camera inside a big mirror sphere: every primary ray hits from inside (far root)."""
    spec = S.readme_spec(48, 27)
    spec["spheres"].append({"center": [0, 0.2, -2], "radius": 0.5,
                            "shader": {"reflection_gain": 0.3, "specular_gain": 0.7, "specular_roughness": 0.3,
                                       "iridescence_gain": 0.08, "diffuse_gain": 0.6,
                                       "texture": {"kind": "const", "color": [0.2, 0.4, 0.9]}}})
    return spec


def no_dome_spec():
    spec = S.main_spec(64, 36)
    spec["lights"] = [{"kind": "point", "position": [1, 3, -1]}]
    return spec


def multi_dome_spec():
    spec = S.readme_spec(64, 36)
    spec["lights"].append({"kind": "dome", "intensity": 0.25, "color": [0.2, 0.5, 1.0]})
    spec["lights"].insert(1, {"kind": "point", "position": [9, 9, 9]})  # not lights[0]: unused
    return spec


def main():
    cases = {
        "main_160x90_B0": (S.main_spec(160, 90), 0),
        "main_160x90_B1": (S.main_spec(160, 90), 1),
        "main_160x90_B3": (S.main_spec(160, 90), 3),
        "main_160x90_B5": (S.main_spec(160, 90), 5),
        "main_160x90_Binf": (S.main_spec(160, 90), None),
        "readme_160x90_B0": (S.readme_spec(160, 90), 0),
        "readme_160x90_B3": (S.readme_spec(160, 90), 3),
        "readme_160x90_Binf": (S.readme_spec(160, 90), None),
        "readme_1x1_B3": (S.readme_spec(1, 1), 3),
        "readme_7x5_B3": (S.readme_spec(7, 5), 3),
        "rand16_128x72_B4": (S.random_spec(16, 0, 128, 72), 4),
        "rand64_96x54_B5": (S.random_spec(64, 0, 96, 54), 5),
        "orbit_k37_rand16_96x54_B3": (S.with_camera(S.random_spec(16, 0, 96, 54), S.orbit_position(37)), 3),
        "ties_64x36_B2": (tie_spec(), 2),
        "inside_48x27_B3": (inside_spec(), 3),
        "nodome_64x36_B3": (no_dome_spec(), 3),
        "multidome_64x36_B3": (multi_dome_spec(), 3),
    }
    arrays = {}
    meta = {
        "numpy": np.__version__,
        "python": sys.version.split()[0],
        "machine": platform.machine(),
        "cpu_flags": _cpu_flags(),
        "note": "Outputs of the reference NumpyRenderer (capped wrapper) run in the build container.",
        "cases": {},
    }
    for name, (spec, B) in cases.items():
        t0 = time.time()
        out, rays, hits, *_ = ref_render(spec, B)
        arrays[name] = out
        meta["cases"][name] = {"spec": spec, "max_bounces": B, "rays": rays, "hits": hits}
        print(f"{name}: {time.time() - t0:.2f}s levels={len(rays)} rays={rays[:6]} hits={hits[:6]}")

    # full-size pins: 1920x1080, B=3, main and README scenes
    for tag, spec in (("main", S.main_spec(1920, 1080)), ("readme", S.readme_spec(1920, 1080))):
        t0 = time.time()
        out, rays, hits, scene, rend, col = ref_render(spec, 3)
        png = HERE / f"ref_1080p_B3_{tag}.png"
        rend.save_image(col, scene.camera, png)
        meta[f"ref_1080p_B3_{tag}"] = {"spec": spec, "max_bounces": 3, "rays": rays, "hits": hits,
                                       "sha256_f64": hashlib.sha256(np.ascontiguousarray(out).tobytes()).hexdigest(),
                                       "max": float(out.max()), "sum": float(out.sum())}
        print(f"1080p {tag}: {time.time() - t0:.2f}s rays={rays} hits={hits}")

    # the reference's committed golden image (main.py, unbounded bounces)
    shutil.copyfile(REF / "render.png", HERE / "render_main_960x540.png")
    meta["render_main_960x540"] = {"spec": S.main_spec(960, 540), "max_bounces": None,
                                   "source": "/root/reference/render.png (== docs/images/render2.png)"}

    np.savez_compressed(HERE / "renders.npz", **arrays)
    (HERE / "scenes.json").write_text(json.dumps(meta, indent=1))

    # intersect known answers (shape.py:28-51)
    V = R["NumpyVector3D"]
    kat = []

    def add(center, radius, O, D, label):
        sph = R["NumpySphere"](V(*center), radius, None)
        d = V(*D).norm() if label != "raw" else V(*D)
        t = sph.intersect(V(*O), V(np.array([d.x], dtype=float), np.array([d.y], dtype=float),
                                      np.array([d.z], dtype=float)))
        kat.append({"center": center, "radius": radius, "origin": O,
                    "dir": [float(np.asarray(d.x).ravel()[0]), float(np.asarray(d.y).ravel()[0]),
                            float(np.asarray(d.z).ravel()[0])],
                    "t": float(np.asarray(t).ravel()[0]), "label": label})

    add([0, 0, 0], 1, [0, 0, -3], [0, 0, 1], "hit front (test_objects.py:6-11)")
    add([0, 0, 0], 1, [0, 0, -3], [0, 1, 1], "miss (test_objects.py:14-19)")
    add([0, 0, 0], 1, [1, 0, -3], [0, 0, 1], "tangent: disc == 0 is a miss")
    add([0, 0, 0], 1, [0, 0, 0], [0, 0, 1], "origin inside: far root")
    add([0, 0, 0], 1, [0, 0, 3], [0, 0, 1], "sphere behind the origin")
    add([0, -99999.5, 0], 99999, [0, 0.2, -2], [0.1, -0.3, 1], "ground sphere R=99999")
    add([0, -99999.5, 0], 99999, [0, 0.2, -2], [0.1, 0.3, 1], "ground sphere, ray upward")
    add([0.55, 0.5, 3], 1.0, [0, 0.2, -2], [0.1, 0.05, 1], "main.py sphere 0")
    add([-0.45, 0.1, 1], 0.4, [0, 0.2, -2], [-0.15, -0.03, 1], "main.py sphere 1")
    # origin exactly on the surface (c == 0) and b = 1.6e-162 > 0: b*b is subnormal and rounds up,
    # so sqrt(disc) > b and the far root is a hit at 3.1e-163 (not "behind the origin")
    add([0, 0, 0], 1, [1, 0, 0], [8e-163, 1, 0], "surface origin, b*b subnormal: tiny hit")
    add([0, 0, 0], 1, [0, 0, -3], [0, 0, 0], "raw")  # zero direction (not normalised)
    (HERE / "intersect_kat.json").write_text(json.dumps(kat, indent=1))

    # NumpyVector3D.norm known answer (intent of test_vectors.py:28-31)
    n = V(3, 4, 0).norm()
    (HERE / "vector_kat.json").write_text(json.dumps({"norm_3_4_0": [n.x, n.y, n.z]}))
    print("done")


def _cpu_flags():
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("flags"):
                fl = line.split(":", 1)[1].split()
                return sorted(f for f in fl if f.startswith("avx512") or f in ("avx2", "fma"))
    except OSError:
        pass
    return []


if __name__ == "__main__":
    main()
