"""The kernels' sin (rtx_kernels.hip sin_reduced, used for the iridescence phase, shader.py:211)
is within 2 ulp of the true sine. NumPy's own SIMD sin is not correctly rounded either (~1 ulp), so
the render parity bar is the colour tolerance of tests/test_gpu_parity.py, not bit equality.

The device function's source is extracted from the .hip file and compiled for the host with gcc
(the same expression sequence, IEEE double with fma, no contraction), then compared with the x87
long-double sinl over the iridescence phase range and beyond, including arguments next to
multiples of pi."""

import re
import shutil
import subprocess

import pytest

from tests.conftest import REPO

HARNESS = r"""
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
%s
static double ulp(double y) { int e; frexp(y, &e); return ldexp(1.0, e - 53); }
int main(void) {
  const double ranges[][2] = {{0.0, 9.42477796076938}, {0.0, 32.0}, {-1000.0, 1000.0}, {0.0, 1048576.0}};
  double worst = 0.0;
  srand48(7);
  for (int k = 0; k < 4; ++k) {
    for (long i = 0; i < 400000; ++i) {
      const double x = ranges[k][0] + (ranges[k][1] - ranges[k][0]) * (i & 1 ? drand48() : (double)i / 400000);
      const long double ref = sinl((long double)x);
      const double u = fabsl((long double)sin_reduced(x) - ref) / ulp((double)ref);
      if (u > worst) worst = u;
    }
  }
  for (int m = 1; m < 20000; ++m) {  /* next to multiples of pi, where x - n*pi cancels */
    double x = m * 3.141592653589793;
    for (int j = 0; j < 16; ++j, x = nextafter(x, 1e300)) {
      const long double ref = sinl((long double)x);
      const double u = fabsl((long double)sin_reduced(x) - ref) / ulp((double)ref);
      if (u > worst) worst = u;
    }
  }
  printf("%%.4f\n", worst);
  return 0;
}
"""


def _device_function():
    src = (REPO / "python_ray_tracer_amd" / "csrc" / "rtx_kernels.hip").read_text()
    m = re.search(r"__device__ __forceinline__ double sin_reduced\(double x\) \{.*?\n\}\n", src, re.S)
    assert m, "sin_reduced not found"
    body = m.group(0).replace("__device__ __forceinline__", "static")
    return body.replace("__builtin_rint", "rint").replace("__builtin_fma", "fma")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_sin_within_two_ulp(tmp_path):
    c = tmp_path / "sin.c"
    c.write_text(HARNESS % _device_function())
    exe = tmp_path / "sin"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    worst = float(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    assert worst <= 2.0, worst
