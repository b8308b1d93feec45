"""A/B patch: hit_color's texture colour by selects instead of branches (k_render_fast, IMG = false)."""


def patch(src: str) -> str:
    old = """  double tr, tg, tb;
  const double tex = mh[RTX_M_TEX];
  if (tex == RTX_TEX_CHECKER) {  // TextureChecker.get_color (:29-32): white * checker
    tr = tg = tb = tk ? 1.0 : 0.0;
  } else if (IMG && tex == RTX_TEX_IMAGE) {"""
    new = """  double tr, tg, tb;
  const double tex = mh[RTX_M_TEX];
  if (!IMG) {
    const bool ck = tex == RTX_TEX_CHECKER;
    const double c = tk ? 1.0 : 0.0;
    tr = ck ? c : (double)mh[RTX_M_TR];
    tg = ck ? c : (double)mh[RTX_M_TG];
    tb = ck ? c : (double)mh[RTX_M_TB];
  } else if (tex == RTX_TEX_CHECKER) {  // TextureChecker.get_color (:29-32): white * checker
    tr = tg = tb = tk ? 1.0 : 0.0;
  } else if (IMG && tex == RTX_TEX_IMAGE) {"""
    assert old in src
    return src.replace(old, new)
