"""A/B patch: the shape's own shadow-ray test (t_self, shader.py:126) evaluated together with the
first pair of the other spheres' tests, one 'any lane may hit' branch for the three square roots
(scenes without a culling tree; bit-identical results)."""


def patch(src: str) -> str:
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
    assert old in src
    src = src.replace(old, new)
    old = """  if (lit && j < nshadow) {
    const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;"""
    new = """  if (lit && j < nshadow) {  // (the loop above breaks with j < nshadow only when lit is false)
    const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;"""
    assert old in src
    return src.replace(old, new)
