"""Ablation (timing only, wrong output): culled scenes skip the shadow walk (lit_bvh)."""

def patch(src: str) -> str:
    old = "  if (culled) lit = lit_bvh(sc, qx, qy, qz, qq, lx, ly, lz, tself, hs, tame, wk);"
    assert old in src
    return src.replace(old, "  // ablation: no shadow walk for culled scenes (timing only)")
