"""A/B patch: the view vector is normalised for every hit (no weighted || need_irid branch)."""


def patch(src: str) -> str:
    old = """  if (weighted || need_irid) {
    double vx = sc[RTX_H_CAM + 0] - px"""
    new = """  {
    double vx = sc[RTX_H_CAM + 0] - px"""
    assert old in src
    return src.replace(old, new)
