"""Scene packer: ``Scene3D`` -> one float64 blob (layout: ``include/rtx_hip.h``).

Everything the reference reads from the scene during a render is flattened
here, once per scene/camera, and uploaded (≈10 KB). Per-material constants that the reference
evaluates in Python scalar arithmetic (``alpha = roughness**2``, ``F0``, the thin-film hue shift,
``1.0/radius``, ``|C|^2``, the level-0 camera terms of ``shape.py:35-37`` …) are evaluated here with
the very same Python expressions, so they are bit-identical to what the reference computes.

Duck-typed: works with this package's ``HipSphere``/``HipShader`` and with the reference's own
``NumpySphere``/``NumpyShader`` objects (same attribute names), so an existing reference scene
renders unchanged.
"""

from __future__ import annotations

import functools
import hashlib

import numpy as np

from . import _lib as L


def _xyz(v):
    return float(v.x), float(v.y), float(v.z)


def _linspace_params(start, stop, num: int):
    """np.linspace(start, stop, num) as (start, step, stop, fix_last): y_i = i*step + start and,
    when num > 1, the last element is set to stop exactly (numpy/_core/function_base.py)."""
    start = float(start)
    stop = float(stop)
    div = num - 1
    if div > 0:
        step = (stop - start) / div
        if step == 0:
            raise NotImplementedError("np.linspace denormal-step branch is not supported")
        return start, step, stop, 1.0
    return start, 0.0, stop, 0.0


def camera_words(position, width: int, height: int) -> dict:
    """get_ray_directions' screen (base.py:123-141) as kernel parameters."""
    if int(width) <= 0 or int(height) <= 0:
        raise ValueError(f"camera size must be positive, got {width}x{height}")
    aspect_ratio = float(width) / height
    screen = (-1, 1 / aspect_ratio + 0.25, 1, -1 / aspect_ratio + 0.25)
    xs = _linspace_params(screen[0], screen[2], int(width))
    ys = _linspace_params(screen[1], screen[3], int(height))
    cx, cy, cz = position
    vz = 0 - cz
    return {"xs": xs, "ys": ys, "vz": vz, "vz2": vz * vz, "oo": (cx * cx + cy * cy) + cz * cz}


def _shape_fields(shape):
    if hasattr(shape, "texture"):
        # NumpyTexturedSphere (shape.py:57-90) passes an RGB colour as its shader and cannot render
        # in the reference either (base.py:110); image textures are out of scope.
        raise NotImplementedError("image-textured spheres are not supported (reference NumpyTexturedSphere is broken)")
    pos = getattr(shape, "position", None) or getattr(shape, "center", None)
    if pos is None or not hasattr(shape, "radius") or not hasattr(shape, "shader"):
        raise TypeError(f"HipRenderer renders spheres only; got {type(shape).__name__}")
    sh = shape.shader
    tex = sh.diffuse_color
    if type(tex).__name__ == "TextureChecker":
        tex_fields = (L.TEX_CHECKER, 1.0, 1.0, 1.0)
    elif hasattr(tex, "texels") and hasattr(tex, "digest"):  # ImageTexture
        tex_fields = (L.TEX_IMAGE, _Texels(tex.texels, tex.digest), float(tex.texels.shape[1]),
                      float(tex.texels.shape[0]))
    elif hasattr(tex, "color"):
        tex_fields = (0.0,) + _xyz(tex.color)
    else:
        raise TypeError(f"unsupported texture {type(tex).__name__}")
    # raw values, not float()-converted: the packer applies the reference's own expressions to them
    return (_xyz(pos), shape.radius, tex_fields, sh.specular_gain, sh.diffuse_gain, sh.specular_roughness,
            sh.specular_ior, sh.iridescence_gain, sh.thin_film_weight, sh.thin_film_thickness, sh.thin_film_ior,
            sh.reflection_gain)


class _Texels:
    """An image texture's texels inside a hashable scene key (hashed by content digest)."""

    __slots__ = ("texels", "digest")

    def __init__(self, texels, digest) -> None:
        self.texels = texels
        self.digest = digest

    def __hash__(self) -> int:
        return hash(self.digest)

    def __eq__(self, other) -> bool:
        return isinstance(other, _Texels) and other.digest == self.digest


def scene_key(scene) -> tuple:
    """Everything a render reads from ``scene`` as a hashable pair
    ``(static, camera)``: ``static`` = per-sphere geometry and material, lights[0].position and
    the DomeLights; ``camera`` = (position, width, height). Raises what the reference raises for
    an unrenderable scene (see pack_scene)."""
    shapes = list(scene.shapes)
    S = len(shapes)
    if S == 0:
        # reduce(np.minimum, []) in NumpyRenderer.raytrace_scene (base.py:98)
        raise TypeError("reduce() of empty iterable with no initial value")
    if S > L.MAX_SPHERES:
        raise ValueError(f"at most {L.MAX_SPHERES} spheres per scene, got {S}")
    lights = list(scene.lights)
    light0 = lights[0]  # IndexError like shader.py:75 when the scene has no light
    lpos = light0.position  # AttributeError like shader.py:75 when lights[0] is a DomeLight
    domes = tuple((_xyz(d.color), float(d.intensity)) for d in lights if type(d).__name__ == "DomeLight")
    if len(domes) > L.MAX_DOMES:
        raise ValueError(f"at most {L.MAX_DOMES} DomeLights, got {len(domes)}")
    cam = scene.camera
    W, H = int(cam.width), int(cam.height)
    if W <= 0 or H <= 0:
        raise ValueError(f"camera size must be positive, got {W}x{H}")
    static = (tuple(_shape_fields(sh) for sh in shapes), _xyz(lpos), domes)
    return static, (_xyz(cam.position), W, H)


def pack_scene(scene) -> np.ndarray:
    """Flatten ``scene`` (shapes, lights, camera) into the float64 blob of include/rtx_hip.h."""
    static, camera = scene_key(scene)
    return pack_key(static, camera)


def pack_key(static: tuple, camera: tuple) -> np.ndarray:
    """The blob of a ``scene_key`` pair: the camera-independent part is built once per distinct
    ``static`` (cached), the camera words are applied to a copy."""
    blob = _pack_static(static).copy()
    _apply_camera(blob, *camera)
    return blob


@functools.lru_cache(maxsize=32)
def _pack_static(static: tuple) -> np.ndarray:
    spheres, lpos, domes = static
    S = len(spheres)
    blob = np.zeros(L.HDR_WORDS + S * (L.GEOM_WORDS + L.MAT_WORDS), dtype=np.float64)
    h = blob[: L.HDR_WORDS]
    h[L.H_MAGIC] = L.MAGIC
    h[L.H_NSPH] = S
    h[L.H_LIGHT:L.H_LIGHT + 3] = lpos
    dome_color = (1.0, 1.0, 1.0)  # shader.py:237
    for i, (color, intensity) in enumerate(domes):
        dome_color = color  # the last DomeLight's colour wins (shader.py:241)
        h[L.H_DOMEI + i] = intensity
    h[L.H_DOMEC:L.H_DOMEC + 3] = dome_color
    h[L.H_NDOME] = len(domes)

    geo_rows, mat_rows = [], []
    for sp in spheres:
        (cx, cy, cz), radius = sp[0], sp[1]
        cc = (cx * cx + cy * cy) + cz * cz  # abs(self.position), shape.py:35
        rr = radius * radius  # shape.py:36
        # G_C0 (camera-dependent) is filled by _apply_camera
        geo_rows.append((cx, cy, cz, cc, rr, 1.0 / radius, 0.0, 0.0))  # 1/r: shader.py:74
        mat_rows.append(_material_row(sp))
    geo = blob[L.HDR_WORDS: L.HDR_WORDS + S * L.GEOM_WORDS].reshape(S, L.GEOM_WORDS)
    geo[:] = np.asarray(geo_rows, dtype=np.float64)
    blob[L.HDR_WORDS + S * L.GEOM_WORDS:] = np.asarray(mat_rows, dtype=np.float64).ravel()
    h[L.H_SINRED] = 1.0 if all(sin_reduced_ok(m) for m in mat_rows) else 0.0
    if S >= BVH_MIN_SPHERES:
        blob = _append_culling_tree(blob, geo.copy(), S)
        if S <= SHGRID_MAX_SPHERES:  # (the kernel reads the grid only with a culling tree)
            blob = _append_shadow_grid(blob, geo.copy(), S, lpos)
    if SBOX_MIN_SPHERES <= S <= SBOX_MAX_SPHERES:  # image-plane boxes, unbounded until _apply_camera fills them
        off = blob.size
        blob = np.concatenate([blob, np.tile([-np.inf, np.inf, -np.inf, np.inf], S)])
        blob[L.H_SBOX] = off
    # image textures: one float64 RGB texel table per distinct image, after everything else; the
    # material's RTX_M_TR word holds its word offset
    textures, offsets, size = [], {}, blob.size
    for s_idx, sp in enumerate(spheres):
        tex = sp[2]
        if tex[0] != L.TEX_IMAGE:
            continue
        ref = tex[1]
        if ref.digest not in offsets:
            offsets[ref.digest] = size
            size += ref.texels.size
            textures.append(ref.texels)
        blob[L.HDR_WORDS + S * L.GEOM_WORDS + s_idx * L.MAT_WORDS + L.M_TR] = offsets[ref.digest]
    if textures:
        blob = np.concatenate([blob] + [t.ravel() for t in textures])
    blob.setflags(write=False)
    return blob


def _material_row(fields) -> list:
    """The RTX_MAT_WORDS material record of one sphere's _shape_fields (an image texture's texel
    table offset, RTX_M_TR, is left 0 for the caller to set once the blob is laid out)."""
    _, _, tex, g, dg, rough, ior, ig, tfw, tft, tfior, refl = fields
    m = [0.0] * L.MAT_WORDS
    m[L.M_G] = g
    m[L.M_DG] = dg
    if tex[0] == L.TEX_IMAGE:
        m[L.M_TEX], m[L.M_TR], m[L.M_TG], m[L.M_TB] = L.TEX_IMAGE, 0.0, tex[2], tex[3]
    else:
        m[L.M_TEX], m[L.M_TR], m[L.M_TG], m[L.M_TB] = tex
    # _calculate_physical_specular constants (shader.py:290-301), same Python expressions
    alpha = rough**2
    F0 = ((ior - 1) / (ior + 1)) ** 2
    m[L.M_A2] = alpha**2
    m[L.M_A2M1] = alpha**2 - 1
    m[L.M_1MA2] = 1 - alpha**2
    m[L.M_F0] = F0
    m[L.M_1MF0] = 1 - F0
    # _calculate_physical_iridescence constants (shader.py:208-232)
    hue_shift = (tfior - 1.0) / 2.0
    m[L.M_IG] = ig
    m[L.M_TFW] = tfw
    m[L.M_TFT] = tft
    m[L.M_HS] = hue_shift
    m[L.M_1MHS] = 1.0 - hue_shift
    m[L.M_ROUGH] = rough
    m[L.M_REFL] = refl
    m[L.M_IOR] = ior
    m[L.M_TFIOR] = tfior
    return m


def sin_reduced_ok(m) -> bool:
    """RTX_H_SINRED for one material record: its thin-film phase ((af * pi) * thickness) * 10 with
    af in [0, 1] (shader.py:204-208) stays inside the kernel sine's reduction range (|x| <= 2^20)."""
    return bool(abs(m[L.M_TFT]) <= L.SIN_TFT_MAX)


def pack_override(scene, shape, shader) -> np.ndarray:
    """The blob of ``scene`` plus a level-0 material record for ``shader`` (RTX_H_MAT0):
    NumpyShader.create called on a shader that is not ``shape``'s own shades the hits with the
    shader's parameters on the shape's geometry (shader.py:73-112 reads ``self.*``), and traces the
    reflections through the unchanged scene (shader.py:152). An image texture's texels are appended
    after the record."""
    import types

    static, camera = scene_key(scene)
    pos = getattr(shape, "position", None) or getattr(shape, "center", None)
    fields = _shape_fields(types.SimpleNamespace(position=pos, radius=shape.radius, shader=shader))
    m = _material_row(fields)
    blob = pack_key(static, camera)
    off = blob.size
    parts = [blob, np.asarray(m, dtype=np.float64)]
    if fields[2][0] == L.TEX_IMAGE:
        parts[1][L.M_TR] = off + L.MAT_WORDS
        parts.append(fields[2][1].texels.ravel())
    out = np.concatenate(parts)
    out[L.H_MAT0] = off
    if not sin_reduced_ok(m):
        out[L.H_SINRED] = 0.0
    return out


def _apply_camera(blob: np.ndarray, cpos, W: int, H: int) -> None:
    """Camera header words and every sphere's level-0 ``c`` (shape.py:35-37 with the camera as the
    ray origin: ((|C|^2 + |O|^2) - 2 C.O) - r^2, elementwise in the reference's order)."""
    h = blob[: L.HDR_WORDS]
    cw = camera_words(cpos, W, H)
    h[L.H_CAM:L.H_CAM + 3] = cpos
    h[L.H_XSTART], h[L.H_XSTEP], h[L.H_XSTOP], h[L.H_XFIX] = cw["xs"]
    h[L.H_YSTART], h[L.H_YSTEP], h[L.H_YSTOP], h[L.H_YFIX] = cw["ys"]
    h[L.H_VZ], h[L.H_VZ2] = cw["vz"], cw["vz2"]
    h[L.H_W], h[L.H_H] = W, H
    h[L.H_CAMOO] = cw["oo"]
    ox, oy, oz = cpos
    S = int(h[L.H_NSPH])
    tables = [blob[L.HDR_WORDS: L.HDR_WORDS + S * L.GEOM_WORDS]]
    if h[L.H_NNODES]:
        tables.append(blob[int(h[L.H_CGEO]): int(h[L.H_CGEO]) + S * L.GEOM_WORDS])
    for t in tables:
        geo = t.reshape(S, L.GEOM_WORDS)
        co = (geo[:, L.G_CX] * ox + geo[:, L.G_CY] * oy) + geo[:, L.G_CZ] * oz
        geo[:, L.G_C0] = ((geo[:, L.G_CC] + cw["oo"]) - 2 * co) - geo[:, L.G_RR]
    h[L.H_TAME] = 1.0 if is_tame(tables[0].reshape(S, L.GEOM_WORDS), cpos) else 0.0
    if h[L.H_SBOX]:
        off = int(h[L.H_SBOX])
        blob[off: off + 4 * S] = sphere_plane_boxes(tables[0].reshape(S, L.GEOM_WORDS), cpos).ravel()


# --- image-plane boxes (RTX_H_SBOX) -----------------------------------------------------------
# A camera ray leaves O through the image-plane point (x, y, 0) (base.py:123-141: direction
# norm(x - Ox, y - Oy, 0 - Oz)). Projected on the xz plane, a ray that comes within R of the centre
# C passes within R of (Cx, Cz) (projection shortens distances), so its plane point's x lies where
# the half-lines from (Ox, Oz) through (x, 0) meet the disc (Cx, Cz; R): between the two tangents'
# crossings of z = 0, both tangent directions heading towards the plane (else unbounded); likewise
# y on the yz plane. R is r plus the doubled culling margin (rtx_kernels.hip wave_frustum), which
# covers the reference root's rounding and the ray direction's normalisation; the box is padded for this function's own rounding and for
# the lane's plane point Ox + fl(x - Ox), within an ulp of x.
# the culled kernels (from BVH_MIN_SPHERES): the small-scene kernels gain nothing from them (A/B r5t,
# r5y-r5zd: C2 +10% with the level-0 tests skipped, however the candidates are built; tools/ab_patches.py
# small_boxes*, packed with SBOX_MIN_SPHERES=1)
SBOX_MIN_SPHERES = 8
SBOX_MAX_SPHERES = 128
SBOX_MIN_TZ = 1e-3  # tangent directions closer than this to the image plane: an unbounded side


def sphere_plane_boxes(geo: np.ndarray, cpos) -> np.ndarray:
    """[S, 4] {x lo, x hi, y lo, y hi}: camera rays through image-plane points outside a sphere's box
    yield FARAWAY for it (NumpySphere.intersect, shape.py:28-51); infinite bounds where none hold."""
    O = np.asarray(cpos, dtype=np.float64)
    C = geo[:, L.G_CX:L.G_CZ + 1]
    rr = geo[:, L.G_RR]
    w = C - O
    scale = ((w * w).sum(axis=1) + 2.0 * geo[:, L.G_CC]) + 3.0 * rr + float(O @ O)
    R = (np.sqrt(rr) + 2e-7 * (scale + 1.0)) * (1.0 + 1e-9)
    vz = 0.0 - O[2]
    out = np.tile(np.array([-np.inf, np.inf, -np.inf, np.inf]), (len(geo), 1))
    if not (vz != 0.0 and np.all(np.isfinite(O))):
        return out
    sg = 1.0 if vz > 0 else -1.0
    with np.errstate(all="ignore"):
        for k, a in enumerate((0, 1)):
            wa, wz = w[:, a], w[:, 2]
            d = np.sqrt(wa * wa + wz * wz)
            ua, uz = wa / d, wz / d
            sa = R / d
            ca = np.sqrt(np.maximum(1.0 - sa * sa, 0.0))
            xs, ok = [], (d > R * (1.0 + 1e-9)) & np.isfinite(d) & np.isfinite(R)
            for sgn in (1.0, -1.0):  # the two tangent directions: u rotated by +-alpha
                ta = ua * ca - sgn * uz * sa
                tz = uz * ca + sgn * ua * sa
                ok &= sg * tz > SBOX_MIN_TZ
                x = O[a] + vz * (ta / tz)
                pad = 1e-9 * (np.abs(x) + abs(O[a]) + 1.0) + 1e-12 * abs(vz) / (tz * tz)
                xs.append((x - pad, x + pad))
            lo = np.minimum(xs[0][0], xs[1][0])
            hi = np.maximum(xs[0][1], xs[1][1])
            ok &= np.isfinite(lo) & np.isfinite(hi)
            out[ok, 2 * k] = lo[ok]
            out[ok, 2 * k + 1] = hi[ok]
    return out


def is_tame(geo: np.ndarray, cpos) -> bool:
    """RTX_H_TAME: every sphere centre coordinate, radius and camera coordinate below 2^60 in
    magnitude (finite). Origins of every later ray then stay below ~2^140 (hits lie closer than
    FARAWAY), which the kernel's half-b sphere test relies on (rtx_kernels.hip, SphTest)."""
    vals = np.concatenate([geo[:, L.G_CX:L.G_CZ + 1].ravel(), 1.0 / geo[:, L.G_INVR],
                           np.asarray(cpos, dtype=np.float64)])
    return bool(np.all(np.abs(vals) < L.TAME_BOUND))


# --- culling hierarchy ----------------------------------------------------------------------
# Scenes with many spheres get a tree of axis-aligned boxes over the small spheres (surface-area
# split, up to BVH_LEAF spheres per leaf: 8 measured best, 6-8 within 0.5%); huge spheres (the R=99999 ground) are tested by every
# ray. The kernel's node test is conservative (margins far above the reference formula's rounding
# error, rtx_kernels.hip node_may_hit), so culling changes no result bit. The tree only reorders
# which spheres a ray examines.
BVH_MIN_SPHERES = 8
BVH_LEAF = 8
HUGE_RADIUS = 100.0
# Split criterion (surface-area heuristic): a node of n spheres is split when
#   node_cost * 2 + (A_left * n_left + A_right * n_right) / A < n   (costs in sphere tests),
# i.e. when testing the two child boxes plus the expected sphere tests behind them is cheaper than
# testing the n spheres; nodes above BVH_LEAF spheres always split. None: split every node above
# BVH_LEAF (round 2's build).
BVH_NODE_COST = None


def _box(centers: np.ndarray, radii: np.ndarray):
    lo = (centers - radii[:, None]).min(axis=0)
    hi = (centers + radii[:, None]).max(axis=0)
    pad = 1e-12 * (np.abs(lo) + np.abs(hi)) + 1e-300  # absorb this computation's own rounding
    return lo - pad, hi + pad


def _area(lo, hi):
    e = np.maximum(hi - lo, 0.0)
    return float(e[0] * e[1] + e[1] * e[2] + e[2] * e[0])


def _sah_split(idx, centers, radii):
    """Best surface-area split of sphere list `idx` (sorted along one axis, prefix/suffix boxes)."""
    best = None
    for axis in range(3):
        order = sorted(idx, key=lambda i: (centers[i][axis], i))
        n = len(order)
        lo_c = centers[order] - radii[order][:, None]
        hi_c = centers[order] + radii[order][:, None]
        pre_lo, pre_hi = np.minimum.accumulate(lo_c), np.maximum.accumulate(hi_c)
        suf_lo = np.minimum.accumulate(lo_c[::-1])[::-1]
        suf_hi = np.maximum.accumulate(hi_c[::-1])[::-1]
        for k in range(1, n):
            cost = _area(pre_lo[k - 1], pre_hi[k - 1]) * k + _area(suf_lo[k], suf_hi[k]) * (n - k)
            if best is None or cost < best[0]:
                best = (cost, order[:k], order[k:])
    return best[1], best[2]


def _append_culling_tree(blob: np.ndarray, geo: np.ndarray, S: int) -> np.ndarray:
    centers = geo[:, L.G_CX:L.G_CZ + 1]
    radii = np.sqrt(geo[:, L.G_RR])
    huge = [i for i in range(S) if radii[i] > HUGE_RADIUS or float(np.abs(centers[i]).max()) > 1e4]
    small = [i for i in range(S) if i not in set(huge)]
    order = list(huge)
    nodes = []

    def rec(idx):
        me = len(nodes)
        nodes.append(None)
        lo, hi = _box(centers[idx], radii[idx])
        c = (lo + hi) * 0.5
        R = float(np.sqrt(((hi - lo) ** 2).sum())) * 0.5
        R = R * (1 + 1e-12) + 1e-12
        cc = (float(np.sqrt((c ** 2).sum())) + R) ** 2
        node = [lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], 0, 0, 0, 2e-7 * (3.0 * cc + R * R + 1.0), 0.0, 0.0]
        split = None
        if len(idx) > 1:
            left, right = _sah_split(idx, centers, radii)
            if len(idx) > BVH_LEAF:
                split = (left, right)
            elif BVH_NODE_COST is not None:
                a = _area(lo, hi)
                al = _area(*_box(centers[left], radii[left]))
                ar = _area(*_box(centers[right], radii[right]))
                if a > 0 and 2 * BVH_NODE_COST + (al * len(left) + ar * len(right)) / a < len(idx):
                    split = (left, right)
        if split is None:
            node[L.N_FIRST] = len(order)
            node[L.N_COUNT] = len(idx)
            order.extend(sorted(idx))
        else:
            nodes[me] = node
            rec(split[0])
            rec(split[1])
        node[L.N_SKIP] = len(nodes)
        nodes[me] = node

    if small:
        rec(small)
    node_arr = np.asarray(nodes, dtype=np.float64).reshape(-1, L.NODE_WORDS)
    cgeo = geo[order].copy()
    cgeo[:, L.G_IDX] = order
    hdr_nodes = blob.size
    hdr_cgeo = hdr_nodes + node_arr.size
    out = np.concatenate([blob, node_arr.ravel(), cgeo.ravel()])
    out[L.H_NNODES] = len(nodes)
    out[L.H_NALWAYS] = len(huge)
    # RTX_H_NBEAM: the huge spheres that end the scene (typically the ground, appended last) are
    # candidates of every tile frustum and reflected-ray beam without a test
    out[L.H_NBEAM] = (max(small) + 1) if small else 0
    if out[L.H_NBEAM] == S:
        out[L.H_NBEAM] = 0
    out[L.H_NODES] = hdr_nodes
    out[L.H_CGEO] = hdr_cgeo
    return out


# --- shadow grid -----------------------------------------------------------------------------
# _calculate_shadow (shader.py:114-128) casts, from the nudged hit point q = p + 1e-4 N, a ray along
# L_dir = norm(light - p) and tests every sphere. Its line passes through q and, since its direction
# is that of light - p, through light + (q - p), within 1e-4 |N| of the light. For a voxel V of a grid
# over the small spheres, every such ray (s > 0) with q in V therefore lies within eps_n of the ray
# from p through the light, p in V's bounding ball grown by eps_n (the kernel only uses the voxel
# masks when every lane has |N|^2 <= 4, so eps_n = 2e-4): within eps_n of the capsule of the segment
# from the ball's centre to the light (radius: the ball's) or of the single cone beyond the light,
# apex at the light, around the directions from the ball to the light. A sphere farther from both
# than its radius plus the reference formula's rounding reach (a root it reports lies within
# lm <= 1.8e-7 (|C| + |q| + r) of the ball, the budget of node_may_hit; 1e-6 (... + 1) here) yields
# FARAWAY or a root <= 0 on every such ray and cannot shadow: the voxel's mask leaves it out.
# Distance of a point at w from the light to the cone of unit axis a and half-angle T:
# |w x a| cos T - (w.a) sin T, or |w| when (w.a) cos T + |w x a| sin T < 0 (behind the apex). Rays from outside the grid whose line misses the small spheres' bounding ball
# (tested per lane in the kernel) can only be shadowed by the huge spheres: the last mask. The grid
# covers the small spheres and, for a light above them, their shadow on the plane of their lowest
# point (where a ground under them is hit), at most 3x their extent.
SHGRID_MAX_SPHERES = 128
# cells along the grid's longest side (cubic cells): the first of these whose grid has at most
# SHGRID_MAX_VOXELS voxels (48: C4 -1.8%, C5 -2%, C3 -0.4% against 32, A/B r5p; 64 no better)
SHGRID_CELLS = (48, 32)
SHGRID_MAX_VOXELS = 1 << 14


def _append_shadow_grid(blob: np.ndarray, geo: np.ndarray, S: int, lpos) -> np.ndarray:
    light = np.asarray(lpos, dtype=np.float64)
    centers = geo[:, L.G_CX:L.G_CZ + 1]
    radii = np.sqrt(geo[:, L.G_RR])
    if not (np.all(np.isfinite(light)) and np.all(np.isfinite(centers)) and np.all(np.isfinite(radii))):
        return blob
    small = [i for i in range(S) if not (radii[i] > HUGE_RADIUS or float(np.abs(centers[i]).max()) > 1e4)]
    if not small:
        return blob
    slo = (centers[small] - radii[small][:, None]).min(axis=0)
    shi = (centers[small] + radii[small][:, None]).max(axis=0)
    ext = float((shi - slo).max())
    pad = 1e-3 * ext + 1e-3  # hit points nudged off the spheres (1e-4) and off a ground they rest on
    lo, hi = slo - pad, shi + pad
    if light[1] > hi[1]:  # the small spheres' shadow on the plane y = lo_y, within 3x their extent
        corners = np.array([[x, y, z] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])])
        f = (light[1] - lo[1]) / (light[1] - corners[:, 1])
        proj = light + (corners - light) * f[:, None]
        mid = (lo + hi) * 0.5
        for ax in (0, 2):
            lo[ax] = max(min(lo[ax], proj[:, ax].min()), mid[ax] - 1.5 * (ext + 2 * pad))
            hi[ax] = min(max(hi[ax], proj[:, ax].max()), mid[ax] + 1.5 * (ext + 2 * pad))
    for cells in ((SHGRID_CELLS,) if np.isscalar(SHGRID_CELLS) else SHGRID_CELLS):
        cell = float((hi - lo).max()) / cells
        dims = np.maximum(np.ceil((hi - lo) / cell), 1).astype(np.int64)
        if int(np.prod(dims)) <= SHGRID_MAX_VOXELS:
            break
    else:
        return blob
    inv = 1.0 / cell
    # voxel boxes (grown by a rounding margin: the kernel's index arithmetic may place q one voxel off
    # at a boundary)
    ix, iy, iz = np.meshgrid(np.arange(dims[0]), np.arange(dims[1]), np.arange(dims[2]), indexing="ij")
    idx = np.stack([ix.ravel(order="F"), iy.ravel(order="F"), iz.ravel(order="F")], axis=1)  # x fastest
    vlo = lo + idx * cell
    vhi = lo + (idx + 1) * cell
    m = (vlo + vhi) * 0.5
    grow = 1e-9 * (np.abs(lo).max() + np.abs(hi).max() + float((hi - lo).max())) + 1e-12
    eps_n = 2e-4
    rho = np.sqrt(((vhi - vlo) ** 2).sum(axis=1)) * 0.5 * (1 + 1e-12) + grow + eps_n
    mv = light - m  # voxel -> light
    D = np.sqrt((mv ** 2).sum(axis=1))
    wide = D <= rho * 1.01  # the voxel (nearly) holds the light: every sphere
    Ds = np.where(wide, 1.0, D)
    a = mv / Ds[:, None]  # the cone's axis, pointing away from the voxel
    sinT = np.minimum(rho / Ds * (1 + 1e-12), 1.0)
    cosT = np.sqrt(np.maximum(1.0 - sinT * sinT, 0.0)) * (1 - 1e-12)
    w = centers - light  # [S, 3]
    # (1) beyond the light: the single cone of apex `light` and axis a
    h = a @ w.T  # [V, S]
    cr = np.cross(a[:, None, :], w[None, :, :])
    dperp = np.sqrt((cr ** 2).sum(axis=2))
    wmag = np.sqrt((w ** 2).sum(axis=1))
    behind_apex = h * cosT[:, None] + dperp * sinT[:, None] < 0.0
    d_cone = np.where(behind_apex, wmag[None, :], dperp * cosT[:, None] - h * sinT[:, None])
    # (2) from the voxel to the light: the capsule of the segment [m, light] and radius rho
    cm = centers[None, :, :] - m[:, None, :]  # [V, S, 3]
    tt = np.clip((cm * mv[:, None, :]).sum(axis=2) / (Ds * Ds)[:, None], 0.0, 1.0)
    d_seg = np.sqrt(((cm - tt[:, :, None] * mv[:, None, :]) ** 2).sum(axis=2))
    qmax = np.sqrt((m ** 2).sum(axis=1)) + rho  # |q| bound per voxel
    cmag = np.sqrt((centers ** 2).sum(axis=1))
    margin = (radii[None, :] * (1 + 1e-12) + 1e-6 * (qmax[:, None] + cmag[None, :] + radii[None, :] + 1.0)
              + eps_n + 1e-9 * (wmag[None, :] + D[:, None] + rho[:, None]))
    may = ~((d_cone > margin) & (d_seg > margin + rho[:, None])) | wide[:, None]
    bits = np.zeros((may.shape[0] + 1, 2), dtype=np.uint64)
    for j in range(S):
        bits[:-1][may[:, j], j >> 6] |= np.uint64(1) << np.uint64(j & 63)
        if j not in small:  # the huge spheres' mask
            bits[-1, j >> 6] |= np.uint64(1) << np.uint64(j & 63)
    cb = (slo + shi) * 0.5
    rb = float(np.sqrt(((shi - slo) ** 2).sum())) * 0.5
    rb = rb * (1 + 1e-12) + 1e-6 * (float(np.sqrt((cb ** 2).sum())) + rb + 1.0) + 1e-12
    rec = np.concatenate([lo, [inv, inv, inv], dims.astype(np.float64), cb, [rb], bits.view(np.float64).ravel()])
    off = blob.size
    out = np.concatenate([blob, rec])
    out[L.H_SHGRID] = off
    return out


def sphere_geometry(center, radius) -> np.ndarray:
    """One RTX_GEOM_WORDS record for rtx_sphere_intersect."""
    cx, cy, cz = center
    g = np.zeros(L.GEOM_WORDS, dtype=np.float64)
    g[L.G_CX:L.G_CZ + 1] = (cx, cy, cz)
    g[L.G_CC] = (cx * cx + cy * cy) + cz * cz
    g[L.G_RR] = radius * radius
    g[L.G_INVR] = 1.0 / radius
    return g


def blob_key(blob: np.ndarray) -> bytes:
    return hashlib.blake2b(blob.tobytes(), digest_size=16).digest()
