"""The A/B patch set: named source rewrites of ``csrc/rtx_kernels.hip`` for ``tools/ab_build.py``.

    python tools/ab_build.py OUT.so --patch NAME[,NAME...]

Each patch is ``f(src) -> src``; it asserts its anchors, so a patch whose anchor left the source
fails loudly instead of building the baseline under another name. Three kinds:

* **variants** — the same output by other instructions; timed against the shipped build by
  ``tools/ab.py`` (which checks the frames are equal);
* **ablations** — timing only, wrong output (what a stage costs);
* **instruments** — the shipped arithmetic plus measurement (``tile_trace``).

Where each experiment's result lives:

| patch | kind | result |
|---|---|---|
| ``inlgen`` | ablation | the general kernel carried behind a never-taken branch: C2 +68% (r2) |
| ``nogen`` / ``tinygen`` | ablation | the tie launch removed / a trivial kernel in its place (r2_ab_variants) |
| ``nolit`` / ``noshadow`` | ablation | no shadow walk in culled scenes / no shadow test (r2_ab_variants) |
| ``pair_nobranch`` | variant | both roots of a sphere pair in every lane: +7..11% (r3f) |
| ``tex_select`` | variant | hit_color's texture colour by selects: within noise (r3f) |
| ``v_always`` | variant | V normalised for every hit: within noise (r3f) |
| ``lv_together`` / ``self_triple`` / ``lv_triple`` | variant | ILP in shade(): r3p, not adopted |
| ``tile_trace`` | instrument | per-tile start/end timestamps of k_render_fast (``tools/tile_trace.py``) |
| ``small_boxes`` .. ``small_boxes8`` | variant / instrument | image-plane box candidates for the small-scene kernels' level-0 rays, five ways (pack with ``@SBOX_MIN_SPHERES=1``): all C2 +10..12%; the mask computed and left unused costs the same, a never-taken pair-skip branch alone +0.7% (r5t, r5y-r5zc) |

(The round-2/3 patches were written against the source of their session; their anchors are kept
as they were, so they document the experiment and re-apply to that revision with ``--rev``.)
"""

from __future__ import annotations


def _sub(src: str, old: str, new: str) -> str:
    if old not in src:
        raise SystemExit(f"ab_patches: anchor not found: {old[:100]!r}")
    return src.replace(old, new)


# ---------------------------------------------------------------------------------------------- ablations
def inlgen(src: str) -> str:
    """k_render_fast carries the general kernel's depth-first path behind a branch that is never
    taken (mode 7): what its registers / scratch cost the fast path."""
    a = "  fast_tile<B, LDS, DEEP, LVL, STATS>(p, blockIdx.x, gridDim.y - 1 - blockIdx.y, true, lds_tab);\n}"
    src = _sub(src, a, a[:-1] + "  if (p.mode == 7) general_tail(p);\n}")
    b = "template <int B, bool LDS, bool DEEP, bool LVL = levels_in_lds<B, LDS, DEEP>(), bool STATS = false>"
    src = _sub(src, b, "__device__ void general_tail(const Params& p);\n" + b)
    c = "__global__ __launch_bounds__(64) void k_render_general(Params p0) {"
    return _sub(src, c, """__device__ void general_tail(const Params& p) {
  Stack S{p.stack, p.n_workers, (int64_t)blockIdx.x * kFastBlock + threadIdx.x};
  double cr, cg, cb;
  trace_general(p, S, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0, cr, cg, cb, -1, -1);
  write_out(p, 0, cr, cg, cb);
}

""" + c)


_GEN_LAUNCH = "  hipLaunchKernelGGL(k_render_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);"


def nogen(src: str) -> str:
    """No tie launch for capped renders (timing only: wrong when a frame has ties)."""
    return _sub(src, _GEN_LAUNCH, "  if (!capped)" + _GEN_LAUNCH[1:])


def tinygen(src: str) -> str:
    """The tie launch replaced by a trivial kernel of the same grid that only reads the counters:
    the cost of a second launch apart from k_render_general's own properties."""
    src = _sub(src, _GEN_LAUNCH, """  if (capped) {
    hipLaunchKernelGGL(k_noop_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);
  } else {
  """ + _GEN_LAUNCH + "\n  }")
    b = "// ------------------------------------------------------------------------------------------\n// boundary helpers"
    return _sub(src, b, """__global__ __launch_bounds__(64) void k_noop_general(Params p) {
  uint32_t* hdr = (uint32_t*)p.ws;
  if (hdr[RTX_WS_COUNT] != 0u && threadIdx.x == 0) hdr[RTX_WS_STATUS] |= 8u;
}

""" + b)


def nolit(src: str) -> str:
    """Culled scenes skip the shadow walk (timing only, wrong output)."""
    return _sub(src, "  if (culled) lit = lit_bvh(sc, qx, qy, qz, qq, lx, ly, lz, tself, hs, tame, wk);",
                "  // ablation: no shadow walk for culled scenes (timing only)")


def noshadow(src: str) -> str:
    """No shadow test at all: lit = true (timing only, wrong output)."""
    src = _sub(src, "  const double tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);",
               "  const double tself = 1.0;  // ablation")
    return _sub(src, "  const int nshadow = culled ? 0 : nsph - (hs < nsph);", "  const int nshadow = 0;  // ablation")


# ---------------------------------------------------------------------------------------------- variants
def pair_nobranch(src: str) -> str:
    """The sphere-pair test computes both roots in every lane (no 'any lane may hit' branch)."""
    old = """__device__ __forceinline__ void isect_pair(const SphTest& a, const SphTest& b, F&& f) {
  if (!a.skip || !b.skip) {
    bool v0, v1;
    const double t0 = isect_sol(a, v0);
    const double t1 = isect_sol(b, v1);
    f(t0, v0, t1, v1);
  }
}"""
    return _sub(src, old, """__device__ __forceinline__ void isect_pair(const SphTest& a, const SphTest& b, F&& f) {
  bool v0, v1;
  const double t0 = isect_sol(a, v0);
  const double t1 = isect_sol(b, v1);
  f(t0, v0, t1, v1);
}""")


def tex_select(src: str) -> str:
    """hit_color's texture colour by selects instead of branches (IMG = false)."""
    old = """  double tr, tg, tb;
  const double tex = mh[RTX_M_TEX];
  if (tex == RTX_TEX_CHECKER) {  // TextureChecker.get_color (:29-32): white * checker
    tr = tg = tb = tk ? 1.0 : 0.0;
  } else if (IMG && tex == RTX_TEX_IMAGE) {"""
    return _sub(src, old, """  double tr, tg, tb;
  const double tex = mh[RTX_M_TEX];
  if (!IMG) {
    const bool ck = tex == RTX_TEX_CHECKER;
    const double c = tk ? 1.0 : 0.0;
    tr = ck ? c : (double)mh[RTX_M_TR];
    tg = ck ? c : (double)mh[RTX_M_TG];
    tb = ck ? c : (double)mh[RTX_M_TB];
  } else if (tex == RTX_TEX_CHECKER) {  // TextureChecker.get_color (:29-32): white * checker
    tr = tg = tb = tk ? 1.0 : 0.0;
  } else if (IMG && tex == RTX_TEX_IMAGE) {""")


def v_always(src: str) -> str:
    """The view vector is normalised for every hit (no weighted || need_irid branch)."""
    return _sub(src, "  if (weighted || need_irid) {\n    double vx = sc[RTX_H_CAM + 0] - px",
                "  {\n    double vx = sc[RTX_H_CAM + 0] - px")


def lv_together(src: str) -> str:
    """V (shader.py:76) normalised beside L (:75), before the shadow test: two square-root /
    division chains in one basic block (bit-identical arithmetic; V computed for every hit)."""
    src = _sub(src, """  double lx = sc[RTX_H_LIGHT + 0] - px, ly = sc[RTX_H_LIGHT + 1] - py, lz = sc[RTX_H_LIGHT + 2] - pz;
  norm3(lx, ly, lz);  // :75
""", """  double lx = sc[RTX_H_LIGHT + 0] - px, ly = sc[RTX_H_LIGHT + 1] - py, lz = sc[RTX_H_LIGHT + 2] - pz;
  double vx = sc[RTX_H_CAM + 0] - px, vy = sc[RTX_H_CAM + 1] - py, vz = sc[RTX_H_CAM + 2] - pz;
  {  // :75 and :76, the two chains interleaved (norm3's range ballot for L, V's core as before)
    const double dl = dot3(lx, ly, lz, lx, ly, lz), dv = dot3(vx, vy, vz, vx, vy, vz);
    double rl, rv;
    if (__ballot(!(dl >= 0x1.0p-600 && dl <= 0x1.0p+600)) == 0) {
      rl = div_core(1.0, sqrt_core(dl));
      rv = inv_mag_shade_v(dv);
    } else {
      rl = inv_mag(dl);
      rv = inv_mag_shade_v(dv);
    }
    lx = lx * rl; ly = ly * rl; lz = lz * rl;
    vx = vx * rv; vy = vy * rv; vz = vz * rv;
  }
""")
    return _sub(src, """  if (weighted || need_irid) {
    double vx = sc[RTX_H_CAM + 0] - px, vy = sc[RTX_H_CAM + 1] - py, vz = sc[RTX_H_CAM + 2] - pz;
    {  // :76 (towards the camera on every level); V only feeds the specular and the iridescence
      const double rv = inv_mag_shade_v(dot3(vx, vy, vz, vx, vy, vz));
      vx = vx * rv;
      vy = vy * rv;
      vz = vz * rv;
    }
    if (weighted)""", "  if (weighted || need_irid) {\n    if (weighted)")


def self_triple(src: str) -> str:
    """The shape's own shadow test (t_self, shader.py:126) evaluated with the first pair of the
    other spheres' tests under one 'any lane may hit' branch (round-3 shade(), r3p)."""
    old = """  const double qq = dot3(qx, qy, qz, qx, qy, qz);
  const double tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);
  wk.test(1);
  bool lit = true;
  // t_self beyond FARAWAY (a hit past the reference's sentinel distance): every missing sphere
  // shadows. The linear loop handles it exactly; the culling tree skips missing spheres, so such
  // a wave takes the linear loop.
  const bool far_self = tself > FARAWAY;
  // The shape's own test is t_self itself (same expression), and t_self < t_self never holds: when
  // every active lane hit the same sphere, the loops skip it (wave-uniform index remap below).
  const int h0 = __builtin_amdgcn_readfirstlane(h);
  const int hs = __ballot(h != h0) == 0 ? h0 : nsph;
  const bool culled = TREE && sc[RTX_H_NNODES] != 0.0 && __ballot(far_self) == 0;
  if (culled) lit = lit_bvh(sc, qx, qy, qz, qq, lx, ly, lz, tself, hs, tame, wk);
  const int nshadow = culled ? 0 : nsph - (hs < nsph);
  int j = 0;
"""
    new = """  const double qq = dot3(qx, qy, qz, qx, qy, qz);
  wk.test(1);
  bool lit = true;
  // The shape's own test is t_self itself (same expression), and t_self < t_self never holds: when
  // every active lane hit the same sphere, the loops skip it (wave-uniform index remap below).
  const int h0 = __builtin_amdgcn_readfirstlane(h);
  const int hs = __ballot(h != h0) == 0 ? h0 : nsph;
  const bool tree_scene = TREE && sc[RTX_H_NNODES] != 0.0;
  const int nlin = nsph - (hs < nsph);
  double tself;
  bool far_self;
  int j = 0;
  bool first_pair_done = false;
  if (!tree_scene && nlin >= 2) {
    // t_self and the first pair of other spheres: three independent chains, one branch
    const int j0 = __builtin_amdgcn_readfirstlane(0 + (0 >= hs));
    const int j1 = __builtin_amdgcn_readfirstlane(1 + (1 >= hs));
    const G* g0 = geo + j0 * RTX_GEOM_WORDS;
    const G* g1 = geo + j1 * RTX_GEOM_WORDS;
    wk.test(2);
    const SphTest as = isect_disc(gh, qx, qy, qz, qq, lx, ly, lz, tame);
    const SphTest a0 = isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame);
    const SphTest a1 = isect_disc(g1, qx, qy, qz, qq, lx, ly, lz, tame);
    tself = FARAWAY;
    bool sh = false;
    if (!as.skip || !a0.skip || !a1.skip) {
      bool vs, v0, v1;
      const double ts = isect_sol(as, vs);
      const double t0 = isect_sol(a0, v0);
      const double t1 = isect_sol(a1, v1);
      if (vs) tself = ts;
      const bool fs = tself > FARAWAY;
      sh = shadows(v0, t0, tself, fs) || shadows(v1, t1, tself, fs);
    }
    far_self = tself > FARAWAY;
    if (sh) lit = false;
    j = 2;
    first_pair_done = true;
  } else {
    tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);
    // t_self beyond FARAWAY (a hit past the reference's sentinel distance): every missing sphere
    // shadows. The linear loop handles it exactly; the culling tree skips missing spheres, so such
    // a wave takes the linear loop.
    far_self = tself > FARAWAY;
  }
  const bool culled = tree_scene && __ballot(far_self) == 0;
  if (culled) lit = lit_bvh(sc, qx, qy, qz, qq, lx, ly, lz, tself, hs, tame, wk);
  const int nshadow = culled ? 0 : nlin;
  if (first_pair_done && !lit) j = nshadow;  // shadowed by the first pair: the loops end here
"""
    src = _sub(src, old, new)
    old = """  if (lit && j < nshadow) {
    const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;"""
    new = """  if (lit && j < nshadow) {  // (the loop above breaks with j < nshadow only when lit is false)
    const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;"""
    return _sub(src, old, new)


def lv_triple(src: str) -> str:
    return self_triple(lv_together(src))


# ---------------------------------------------------------------------------------------------- instruments
TRACE_WORDS = 4  # per record: t_start, t_end (s_memrealtime, 100 MHz), tile id, hw id | xcc id << 32


def tile_trace(src: str) -> str:
    """Per-tile timestamps of k_render_fast: every wave records (start, end, tile, hardware id) of
    each tile it renders into a device buffer registered with ``rtx_trace_set(buf)`` (word 1: capacity,
    records from word 8, record k = tile k / wave k of the launch; an unrendered slot stays 0). The
    persistent loop times each fetched tile; the one-tile-per-block path times the wave from kernel entry (scene staging included).
    s_memrealtime is the 100 MHz constant clock; the arithmetic of the render is unchanged."""
    src = _sub(src, "  int no_general;  // RTX_F_NO_GENERAL: no general kernel follows, so nothing may be deferred\n};",
               "  int no_general;  // RTX_F_NO_GENERAL: no general kernel follows, so nothing may be deferred\n"
               "  unsigned long long* trace;  // tile_trace instrument\n};")
    rec = """
__device__ __forceinline__ void trace_rec(const Params& p, unsigned long long t0, unsigned long long id,
                                          unsigned long long slot) {
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (p.trace && (threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
    // one record per tile at its own slot: no shared counter (a global atomic per tile serialised
    // the traced launch across XCDs, ~50 ns per record, 14x the untraced C4 kernel)
    const unsigned long long k = slot;
    if (k < p.trace[1]) {
      unsigned long long* r = p.trace + 8 + 4 * k;
      r[0] = t0; r[1] = t1; r[2] = id; r[3] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    }
  }
}
"""
    anchor = "// TP: 0 = no culling tree and no persistent launch"
    src = _sub(src, anchor, rec + "\n" + anchor)
    src = _sub(src, "  const Params p = frame_view(p0, blockIdx.z);  // frame of a multi-frame launch (grid z)\n",
               "  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();\n"
               "  const Params p = frame_view(p0, blockIdx.z);  // frame of a multi-frame launch (grid z)\n")
    old = ("      fast_tile<B, LDS, DEEP, LVL, STATS, TREE, BEAM>(p, t - row * p.n_tiles_x, p.n_tiles_y - 1 - row, "
           "false, lds_tab, true);\n")
    src = _sub(src, old, "      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();\n" + old +
               "      trace_rec(p, t0, (unsigned long long)t | ((unsigned long long)pw << 32), (unsigned long long)t);\n")
    old = "  fast_tile<B, LDS, DEEP, LVL, STATS, TREE, BEAM>(p, blockIdx.x, gridDim.y - 1 - blockIdx.y, true, lds_tab);\n}"
    src = _sub(src, old, old[:-1] + "  trace_rec(p, t_entry, ((unsigned long long)(blockIdx.y * gridDim.x + blockIdx.x) * "
               "kFastWaves + (threadIdx.x >> 6)) | (1ull << 63), (unsigned long long)(blockIdx.y * gridDim.x + "
               "blockIdx.x) * kFastWaves + (threadIdx.x >> 6));\n}")
    src = _sub(src, "int run_render(Params& p, void* workspace, size_t workspace_bytes, hipStream_t s, bool no_general = false) {\n",
               "unsigned long long* g_trace = nullptr;\n"
               "int run_render(Params& p, void* workspace, size_t workspace_bytes, hipStream_t s, bool no_general = false) {\n"
               "  p.trace = g_trace;\n")
    return _sub(src, "const char* rtx_last_error(void) { return g_err; }\n",
                "const char* rtx_last_error(void) { return g_err; }\n\n"
                "int rtx_trace_set(void* buf) {\n  g_trace = (unsigned long long*)buf;\n  return RTX_OK;\n}\n")


def persist_plain(src: str) -> str:
    """The persistent loop (TP 2) without the learnt order and the per-tile cost records: the fixed
    c + k * n_fetch tiles, no timestamps live across the tile."""
    src = _sub(src, "const int t = order ? (int)order[c + k * nc] : c + k * nc;", "const int t = c + k * nc;")
    src = _sub(src, "const uint64_t tc0 = p.tile_cost ? __builtin_amdgcn_s_memrealtime() : 0;\n", "")
    return _sub(src, "if (p.tile_cost && lane == 0) p.tile_cost[t] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - tc0);\n",
                "")


def block_plain(src: str) -> str:
    """One-tile-per-block launches (TP 0, 1) without the learnt order and the cost records."""
    src = _sub(src, "const uint64_t t_entry = p0.tile_cost ? __builtin_amdgcn_s_memrealtime() : 0;", "")
    src = _sub(src, "  if (p.tile_order) {\n    tb =", "  if (false) {\n    tb =")
    return _sub(src, "  if (p.tile_cost && (threadIdx.x & 63) == 0)  // the block's time: the slowest of its waves\n"
                "    atomicMax(p.tile_cost + tb, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_entry));\n", "")


# ---------------------------------------------------------------------------------------------- round 5
def nu_select(src: str) -> str:
    """nearest_update by selects (no exec-mask branches): the same tmin / hit / tie."""
    old = """  if (valid && t < tmin) {
    tmin = t;
    hit = s;
    tie = false;
  } else if (valid && t == tmin) {
    tie = true;
  }
}"""
    new = """  const bool lt = valid && t < tmin;
  const bool eq = valid && t == tmin;
  tie = lt ? false : (tie || eq);
  hit = lt ? s : hit;
  tmin = lt ? t : tmin;
}"""
    return _sub(src, old, new)


def abl_noshadow_small(src: str) -> str:
    """Ablation (wrong output): scenes below kTreeMinSpheres test no shadow ray (every hit lit)."""
    return _sub(src, "    const int nshadow = nsph - (hs < nsph);\n    double tsh = FARAWAY;",
                "    const int nshadow = 0;  // ablation\n    double tsh = FARAWAY;")


def abl_nospec(src: str) -> str:
    """Ablation (wrong output): the physical specular is not evaluated (0); V still is (iridescence)."""
    return _sub(src, "    if (weighted) spec = specular(mh, g, nx, ny, nz, lx, ly, lz, vx, vy, vz);",
                "    if (weighted) spec = 0.0;  // ablation")


def abl_noirid(src: str) -> str:
    """Ablation (wrong output): no thin-film iridescence term (nor V where only it needs V)."""
    src = _sub(src, "  const bool need_irid = mh[RTX_M_IG] != 0.0;", "  const bool need_irid = false;  // ablation")
    return _sub(src, "  if (igain != 0.0) {", "  if (false) {  // ablation")


def shade_fma(src: str) -> str:
    """Multiply-adds of the shading-only arithmetic (specular, colour terms, iridescence, the forward
    fold) as fused fmas: a few ulp of colour (no hit, shadow, checker or reflection decision reads
    them), one rounding and one instruction fewer each."""
    subs = [
        ("  const double F = mh[RTX_M_F0] + mh[RTX_M_1MF0] * pow5(1.0 - VdotH);  // :291",
         "  const double F = __builtin_fma(mh[RTX_M_1MF0], pow5(1.0 - VdotH), mh[RTX_M_F0]);  // :291"),
        ("  const double denom = (NdotH * NdotH) * mh[RTX_M_A2M1] + 1.0;  // :295",
         "  const double denom = __builtin_fma(NdotH * NdotH, mh[RTX_M_A2M1], 1.0);  // :295"),
        ("  const double Dd = RTX_PI * ((denom * denom) + 1e-8);  // :296",
         "  const double Dd = RTX_PI * __builtin_fma(denom, denom, 1e-8);  // :296"),
        ("  const double dL = (NdotL + sqrt_shade(a2 + oma2 * (NdotL * NdotL))) + 1e-8;  // :299-301",
         "  const double dL = (NdotL + sqrt_shade(__builtin_fma(oma2, NdotL * NdotL, a2))) + 1e-8;  // :299-301"),
        ("  const double dV = (NdotV + sqrt_shade(a2 + oma2 * (NdotV * NdotV))) + 1e-8;",
         "  const double dV = (NdotV + sqrt_shade(__builtin_fma(oma2, NdotV * NdotV, a2))) + 1e-8;"),
        ("div_shade(1.0, Dd * ((4.0 * NdotV) + 1e-8));  // :306",
         "div_shade(1.0, Dd * __builtin_fma(4.0, NdotV, 1e-8));  // :306"),
        ("  const double sf = spec_base + g * glint;  // :315",
         "  const double sf = __builtin_fma(g, glint, spec_base);  // :315"),
        ("  const double ar = (0.004 + ((tr * dli) * litf) * dg) + sc[RTX_H_DOMEC + 0] * di;",
         "  const double ar = __builtin_fma(sc[RTX_H_DOMEC + 0], di, __builtin_fma((tr * dli) * litf, dg, 0.004));"),
        ("  const double ag = (0.004 + ((tg * dli) * litf) * dg) + sc[RTX_H_DOMEC + 1] * di;",
         "  const double ag = __builtin_fma(sc[RTX_H_DOMEC + 1], di, __builtin_fma((tg * dli) * litf, dg, 0.004));"),
        ("  const double ab = (0.004 + ((tb * dli) * litf) * dg) + sc[RTX_H_DOMEC + 2] * di;",
         "  const double ab = __builtin_fma(sc[RTX_H_DOMEC + 2], di, __builtin_fma((tb * dli) * litf, dg, 0.004));"),
        ("    const double r = (ip * hs) + (omhs * (1.0 - ip));  // :221",
         "    const double r = __builtin_fma(ip, hs, omhs * (1.0 - ip));  // :221"),
        ("    const double gg = (ip * omhs) + (hs * (1.0 - ip));  // :222",
         "    const double gg = __builtin_fma(ip, omhs, hs * (1.0 - ip));  // :222"),
        ("    const double b = 0.5 + 0.5 * ip;  // :223", "    const double b = __builtin_fma(0.5, ip, 0.5);  // :223"),
        ("      cr = cr + thr * lr_;\n      cg = cg + thr * lg_;\n      cb = cb + thr * lb_;",
         "      cr = __builtin_fma(thr, lr_, cr);\n      cg = __builtin_fma(thr, lg_, cg);\n      cb = __builtin_fma(thr, lb_, cb);"),
    ]
    for a, b in subs:
        src = _sub(src, a, b)
    return src


def abl_noshadow_tree(src: str) -> str:
    """Ablation (wrong output): culled scenes (TREE kernels) test no shadow ray (every hit lit)."""
    return _sub(src, "  if (TREE && sc[RTX_H_SHGRID] != 0.0 && sc[RTX_H_TAME] != 0.0 &&",
                "  if (TREE) {  // ablation\n  } else if (TREE && sc[RTX_H_SHGRID] != 0.0 && sc[RTX_H_TAME] != 0.0 &&")


def var_nogrid(src: str) -> str:
    """Variant (same output): no shadow-grid lookup; culled scenes' shadow rays walk the tree."""
    return _sub(src, "  if (TREE && sc[RTX_H_SHGRID] != 0.0 && sc[RTX_H_TAME] != 0.0 &&",
                "  if (false && TREE && sc[RTX_H_SHGRID] != 0.0 && sc[RTX_H_TAME] != 0.0 &&")


def var_nobeam(src: str) -> str:
    """Variant (same output): reflected rays walk the culling tree (no wave beam)."""
    return _sub(src, "      if (BEAM && sc[RTX_H_TAME] != 0.0 && wave_beam(", "      if (false && BEAM && sc[RTX_H_TAME] != 0.0 && wave_beam(")


def var_nofrustum(src: str) -> str:
    """Variant (same output): camera rays walk the culling tree (no per-tile frustum candidates)."""
    return _sub(src, "      fr = wave_frustum(p, __builtin_amdgcn_readfirstlane(col - lane % kWaveW),",
                "      fr = false && wave_frustum(p, __builtin_amdgcn_readfirstlane(col - lane % kWaveW),")


def abl_hoist_geo(src: str) -> str:
    """Ablation (wrong output): the sphere loops of nearest_hit and of the small scenes' shadow test
    read sphere 0's geometry every iteration (loop-invariant scalar loads, hoisted): what the scalar
    loads' latency costs those loops."""
    src = src.replace("    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;",
                      "    const P* g0 = geo;  // ablation")
    src = _sub(src, "      const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;\n"
                    "      const G* g1 = geo + __builtin_amdgcn_readfirstlane(j + 1 + (j + 1 >= hs)) * RTX_GEOM_WORDS;",
               "      const G* g0 = geo;  // ablation\n      const G* g1 = geo + RTX_GEOM_WORDS;")
    return src


def nobehind(src: str) -> str:
    """Variant (same output): the 'sphere behind the origin' test leaves the skip flag; the root's
    own sign test (valid: s1 > 0, implied false there) decides alone, two compares fewer per test."""
    src = _sub(src, "    t.skip = !(t.d > 0.0) || (h > 0.0 && c >= 0.0);", "    t.skip = !(t.d > 0.0);")
    return _sub(src, "    t.skip = !(t.d > 0.0) || behind(b, c);", "    t.skip = !(t.d > 0.0);")


def spec_onercp(src: str) -> str:
    """Variant (a few ulp): the specular's G and spec_base share one reciprocal."""
    return _sub(src, """  const double G = ((2.0 * NdotL) * (2.0 * NdotV)) * div_shade(1.0, dL * dV);  // :303
  const double spec_base = ((F * a2) * G) * div_shade(1.0, Dd * __builtin_fma(4.0, NdotV, 1e-8));  // :306""",
                """  const double spec_base = ((F * a2) * ((2.0 * NdotL) * (2.0 * NdotV))) *
                           div_shade(1.0, (dL * dV) * (Dd * __builtin_fma(4.0, NdotV, 1e-8)));  // :303-306""")


def tk_early(src: str) -> str:
    """Variant (same output): the hit's texture key (checker cell / texel) right after P, so that P
    is dead across the shadow test and the specular (fewer live registers there)."""
    old_tail = """  const double tex = mh[RTX_M_TEX];
  s.tk = tex == RTX_TEX_CHECKER ? (trunc_parity(px * 2.0) == trunc_parity(pz * 2.0))  // :30
         : tex != RTX_TEX_IMAGE ? 0
         : IMG ? image_texel(mh, gh, px, py, pz) : -1;  // -1: an untextured k_render_fast build defers the ray
"""
    src = _sub(src, old_tail, "")
    anchor = "  const double px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;  // :73\n"
    return _sub(src, anchor, anchor + old_tail)


def small_boxes(src: str) -> str:
    """Variant (same output): the image-plane box candidates (RTX_H_SBOX) also for the small-scene
    kernels' level-0 rays (pack with SBOX_MIN_SPHERES=1)."""
    src = _sub(src, """__device__ __forceinline__ bool wave_frustum(const Params& p, int c0, int lr0, uint64_t& m0, uint64_t& m1) {
  const cdouble* sc = (const cdouble*)p.scene;
  const int W = p.width;
  if (c0 >= W || lr0 >= p.n_rows) return false;  // no pixel of this wave lies in the frame
  const int c1 = c0 + kWaveW - 1 < W - 1 ? c0 + kWaveW - 1 : W - 1;
  const int l1 = lr0 + kWaveH - 1 < p.n_rows - 1 ? lr0 + kWaveH - 1 : p.n_rows - 1;""",
               """template <int TW = kWaveW, int TH = kWaveH>
__device__ __forceinline__ bool wave_frustum(const Params& p, int c0, int lr0, uint64_t& m0, uint64_t& m1) {
  const cdouble* sc = (const cdouble*)p.scene;
  const int W = p.width;
  if (c0 >= W || lr0 >= p.n_rows) return false;  // no pixel of this wave lies in the frame
  const int c1 = c0 + TW - 1 < W - 1 ? c0 + TW - 1 : W - 1;
  const int l1 = lr0 + TH - 1 < p.n_rows - 1 ? lr0 + TH - 1 : p.n_rows - 1;""")
    src = _sub(src, """  if constexpr (TREE) {
    if (cam0 && nsph <= 128 && sc[RTX_H_NNODES] != 0.0 && sc[RTX_H_SBOX] != 0.0 && sc[RTX_H_TAME] != 0.0 &&
        sc[RTX_H_VZ] != 0.0) {
      const int lane = threadIdx.x & 63;
      fr = wave_frustum(p, __builtin_amdgcn_readfirstlane(col - lane % kWaveW),
                        __builtin_amdgcn_readfirstlane(lr - lane / kWaveW), fm0, fm1);
    }
  }""", """  if constexpr (TREE) {
    if (cam0 && nsph <= 128 && sc[RTX_H_NNODES] != 0.0 && sc[RTX_H_SBOX] != 0.0 && sc[RTX_H_TAME] != 0.0 &&
        sc[RTX_H_VZ] != 0.0) {
      const int lane = threadIdx.x & 63;
      fr = wave_frustum(p, __builtin_amdgcn_readfirstlane(col - lane % kWaveW),
                        __builtin_amdgcn_readfirstlane(lr - lane / kWaveW), fm0, fm1);
    }
  } else {
    if (cam0 && sc[RTX_H_SBOX] != 0.0 && sc[RTX_H_TAME] != 0.0 && sc[RTX_H_VZ] != 0.0) {
      constexpr int TW = wave_w<false>();
      const int lane = threadIdx.x & 63;
      fr = wave_frustum<TW, 64 / TW>(p, __builtin_amdgcn_readfirstlane(col - lane % TW),
                                     __builtin_amdgcn_readfirstlane(lr - lane / TW), fm0, fm1);
    }
  }""")
    src = _sub(src, """    } else if (cam0) {
      nearest_hit<true>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    }
  }
  if constexpr (LDS) {""", """    } else if (fr) {
      nearest_masked<true>(geo, fm0, 0ull, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else if (cam0) {
      nearest_hit<true>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    }
  }
  if constexpr (LDS) {""")
    return src


def small_boxes2(src: str) -> str:
    """Variant (same output): small_boxes with the tile's candidate mask built by a wave-uniform loop
    over the spheres' boxes through the scalar cache (no per-lane global load at the wave's start)."""
    src = small_boxes(src)
    src = _sub(src, """      fr = wave_frustum<TW, 64 / TW>(p, __builtin_amdgcn_readfirstlane(col - lane % TW),
                                     __builtin_amdgcn_readfirstlane(lr - lane / TW), fm0, fm1);""",
               """      const int c0 = __builtin_amdgcn_readfirstlane(col - lane % TW);
      const int lr0 = __builtin_amdgcn_readfirstlane(lr - lane / TW);
      const int W = p.width, H = p.height;
      if (c0 < W && lr0 < p.n_rows) {
        const int c1 = c0 + TW - 1 < W - 1 ? c0 + TW - 1 : W - 1;
        const int l1 = lr0 + 64 / TW - 1 < p.n_rows - 1 ? lr0 + 64 / TW - 1 : p.n_rows - 1;
        auto xv = [&](int c) {
          return (sc[RTX_H_XFIX] != 0.0 && c == W - 1) ? sc[RTX_H_XSTOP] : (double)c * sc[RTX_H_XSTEP] + sc[RTX_H_XSTART];
        };
        auto yv = [&](int r) {
          return (sc[RTX_H_YFIX] != 0.0 && r == H - 1) ? sc[RTX_H_YSTOP] : (double)r * sc[RTX_H_YSTEP] + sc[RTX_H_YSTART];
        };
        const double xa = xv(c0), xb = xv(c1), ya = yv(global_row(p, lr0)), yb = yv(global_row(p, l1));
        const double xlo = __builtin_fmin(xa, xb), xhi = __builtin_fmax(xa, xb);
        const double ylo = __builtin_fmin(ya, yb), yhi = __builtin_fmax(ya, yb);
        const cdouble* bxs = sc + (int)sc[RTX_H_SBOX];
        uint64_t m = 0;
        for (int s = 0; s < nsph; ++s) {
          const cdouble* e = bxs + 4 * s;
          if (!(e[1] < xlo || e[0] > xhi || e[3] < ylo || e[2] > yhi)) m |= uint64_t(1) << s;
        }
        fm0 = m;
        fr = true;
      }""")
    return src


def small_boxes3(src: str) -> str:
    """Variant (same output): small_boxes2's mask, but the level-0 loop keeps nearest_hit's pair
    structure and skips a pair (wave-uniform branch) when neither sphere is a candidate."""
    src = small_boxes2(src)
    src = _sub(src, """    } else if (fr) {
      nearest_masked<true>(geo, fm0, 0ull, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else if (cam0) {""", """    } else if (cam0) {""")
    src = _sub(src, """    } else if (cam0) {
      nearest_hit<true>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    }
  }
  if constexpr (LDS) {""", """    } else if (cam0) {
      nearest_hit<true>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk, fr ? fm0 : ~0ull);
    } else {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    }
  }
  if constexpr (LDS) {""")
    src = _sub(src, """                                            double dy, double dz, double& tmin, int& hit, bool& tie, double tame,
                                            Wk& wk) {
  wk.test(nsph);""", """                                            double dy, double dz, double& tmin, int& hit, bool& tie, double tame,
                                            Wk& wk, uint64_t cand = ~0ull) {
  wk.test(nsph);""")
    src = _sub(src, """  for (; s + 1 < nsph; s += 2) {
    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;
    const P* g1 = g0 + RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)""", """  for (; s + 1 < nsph; s += 2) {
    if (((cand >> s) & 3ull) == 0) continue;  // neither sphere of the pair can be hit (wave-uniform)
    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;
    const P* g1 = g0 + RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)""")
    src = _sub(src, """  if (s < nsph) {
    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s, tmin, hit, tie); });
  }
}""", """  if (s < nsph && ((cand >> s) & 1ull)) {
    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s, tmin, hit, tie); });
  }
}""")
    return src


def small_boxes4(src: str) -> str:
    """Instrument: small_boxes3 with the mask computed but every pair tested (what the mask costs)."""
    src = small_boxes3(src)
    return _sub(src, "tmin, hit, tie, tame, wk, fr ? fm0 : ~0ull);", "tmin, hit, tie, tame, wk, fr ? (fm0 | ~0ull) : ~0ull);")


def small_boxes5(src: str) -> str:
    """Instrument: small_boxes3 without the mask (fr never set), only the pair-skip branch compiled."""
    src = small_boxes3(src)
    return _sub(src, """        fm0 = m;
        fr = true;""", """        fm0 = m;
        fr = m == 0x123456789ull;""")


def small_boxes6(src: str) -> str:
    """Variant (same output): small_boxes2's mask turned into a packed list of the candidates' indices
    (4 bits each, scene order); the level-0 loop keeps nearest_hit's pair shape over that list."""
    src = small_boxes2(src)
    src = _sub(src, """    } else if (fr) {
      nearest_masked<true>(geo, fm0, 0ull, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else if (cam0) {""", """    } else if (fr) {
      nearest_list(geo, fm0, (int)fm1, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else if (cam0) {""")
    src = _sub(src, """        fm0 = m;
        fr = true;""", """        uint64_t lst = 0;
        int k = 0;
        for (int s = 0; s < nsph; ++s) {
          if ((m >> s) & 1ull) {
            lst |= (uint64_t)s << (4 * k);
            ++k;
          }
        }
        fm0 = lst;
        fm1 = (uint64_t)k;
        fr = true;""")
    src = _sub(src, """// (x)^5 and (x)^2.5 for x in [0, 1]""", """// level-0 nearest hit over a packed candidate list (4-bit sphere indices in scene order, k of them)
template <typename P, typename Wk>
__device__ __forceinline__ void nearest_list(const P* geo, uint64_t lst, int k, double ox, double oy, double oz,
                                             double dx, double dy, double dz, double& tmin, int& hit, bool& tie,
                                             double tame, Wk& wk) {
  wk.test(k);
  tmin = FARAWAY;
  hit = -1;
  tie = false;
  int j = 0;
  for (; j + 1 < k; j += 2) {
    const int s0 = __builtin_amdgcn_readfirstlane((int)((lst >> (4 * j)) & 15));
    const int s1 = __builtin_amdgcn_readfirstlane((int)((lst >> (4 * j + 4)) & 15));
    const P* g0 = geo + s0 * RTX_GEOM_WORDS;
    const P* g1 = geo + s1 * RTX_GEOM_WORDS;
    const SphTest a0 = isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame);
    const SphTest a1 = isect_disc_cam(g1, ox, oy, oz, dx, dy, dz, tame);
    isect_pair(a0, a1, [&](double t0, bool v0, double t1, bool v1) {
      nearest_update(v0, t0, s0, tmin, hit, tie);
      nearest_update(v1, t1, s1, tmin, hit, tie);
    });
  }
  if (j < k) {
    const int s0 = __builtin_amdgcn_readfirstlane((int)((lst >> (4 * j)) & 15));
    const SphTest a0 = isect_disc_cam(geo + s0 * RTX_GEOM_WORDS, ox, oy, oz, dx, dy, dz, tame);
    isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s0, tmin, hit, tie); });
  }
}

// (x)^5 and (x)^2.5 for x in [0, 1]""")
    return src


def small_boxes7(src: str) -> str:
    """Instrument: only nearest_hit's pair-skip branch, with a candidate mask of all ones the
    compiler cannot see (no box mask computed)."""
    src = small_boxes3(src)
    src = _sub(src, "tmin, hit, tie, tame, wk, fr ? fm0 : ~0ull);",
               "tmin, hit, tie, tame, wk, ~(uint64_t)(p.width == -5));")
    return src


def small_boxes8(src: str) -> str:
    """Instrument: the box mask computed (kept live through an opaque test) and nothing skipped."""
    src = small_boxes3(src)
    src = _sub(src, "tmin, hit, tie, tame, wk, fr ? fm0 : ~0ull);",
               "tmin, hit, tie, tame, wk, ~0ull);\n      if (fr && fm0 == 0x123456789ull) tmin = 0.0;")
    return src


PATCHES = {f.__name__: f for f in (small_boxes8, small_boxes7, small_boxes6, small_boxes5, small_boxes4, small_boxes3, small_boxes2, small_boxes, tk_early, nobehind, spec_onercp, abl_hoist_geo, abl_noshadow_tree, var_nogrid, var_nobeam, var_nofrustum, shade_fma, abl_noshadow_small, abl_nospec, abl_noirid, nu_select, inlgen, nogen, tinygen, nolit, noshadow, pair_nobranch, tex_select, v_always,
                                   lv_together, self_triple, lv_triple, tile_trace, persist_plain, block_plain)}


def apply(src: str, names: str) -> str:
    for name in [n for n in names.split(",") if n]:
        if name not in PATCHES:
            raise SystemExit(f"unknown patch {name!r}; known: {', '.join(PATCHES)}")
        src = PATCHES[name](src)
    return src
