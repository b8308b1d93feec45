"""Ablation (timing only, wrong output): no shadow test at all (no t_self, no occluder tests): lit = true."""


def patch(src: str) -> str:
    old = "  const double tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);"
    assert old in src
    src = src.replace(old, "  const double tself = 1.0;  // ablation")
    old = "  const int nshadow = culled ? 0 : nsph - (hs < nsph);"
    assert old in src
    return src.replace(old, "  const int nshadow = 0;  // ablation")
