"""A/B patch: the sphere-pair test computes both roots in every lane (no 'any lane may hit' branch)."""


def patch(src: str) -> str:
    old = """__device__ __forceinline__ void isect_pair(const SphTest& a, const SphTest& b, F&& f) {
  if (!a.skip || !b.skip) {
    bool v0, v1;
    const double t0 = isect_sol(a, v0);
    const double t1 = isect_sol(b, v1);
    f(t0, v0, t1, v1);
  }
}"""
    new = """__device__ __forceinline__ void isect_pair(const SphTest& a, const SphTest& b, F&& f) {
  bool v0, v1;
  const double t0 = isect_sol(a, v0);
  const double t1 = isect_sol(b, v1);
  f(t0, v0, t1, v1);
}"""
    assert old in src
    return src.replace(old, new)
