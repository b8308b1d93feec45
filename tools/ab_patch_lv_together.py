"""A/B patch: V (shader.py:76) normalised beside L (:75), before the shadow test: the two square
root / division chains in one basic block (bit-identical arithmetic; V computed for every hit)."""


def patch(src: str) -> str:
    old = """  double lx = sc[RTX_H_LIGHT + 0] - px, ly = sc[RTX_H_LIGHT + 1] - py, lz = sc[RTX_H_LIGHT + 2] - pz;
  norm3(lx, ly, lz);  // :75
"""
    new = """  double lx = sc[RTX_H_LIGHT + 0] - px, ly = sc[RTX_H_LIGHT + 1] - py, lz = sc[RTX_H_LIGHT + 2] - pz;
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
"""
    assert old in src
    src = src.replace(old, new)
    old = """  if (weighted || need_irid) {
    double vx = sc[RTX_H_CAM + 0] - px, vy = sc[RTX_H_CAM + 1] - py, vz = sc[RTX_H_CAM + 2] - pz;
    {  // :76 (towards the camera on every level); V only feeds the specular and the iridescence
      const double rv = inv_mag_shade_v(dot3(vx, vy, vz, vx, vy, vz));
      vx = vx * rv;
      vy = vy * rv;
      vz = vz * rv;
    }
    if (weighted)"""
    new = """  if (weighted || need_irid) {
    if (weighted)"""
    assert old in src
    return src.replace(old, new)
