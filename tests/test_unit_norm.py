"""The closed form the kernels use to re-normalise an already-unit vector (rtx_kernels.hip,
inv_mag_near1) equals the reference's correctly rounded ``1.0 / sqrt(d)`` chain
(NumpyVector3D.norm, ray_tracer/infrastructure/numpy/base.py:61-64) for every squared length d
within 2^-30 of 1: checked exhaustively against IEEE sqrt and division on the host. (The device
side of the same closed form is checked in tests/test_gpu_parity.py::test_fast_sqrt_div_bit_exact.)"""

import numpy as np


def closed_form(d):
    # r = 1 - floor((d - 1) * 2^51) * 2^-52   (every step exact for |d - 1| <= 2^-30)
    return 1.0 - np.floor((d - 1.0) * 2.0 ** 51) * 2.0 ** -52


def test_inv_mag_near1_exhaustive():
    # every double in [1 - 2^-30, 1 + 2^-30]: below 1 the spacing is 2^-53, above it 2^-52
    lim = 1 << 23
    below = 1.0 - np.arange(0, lim + 1, dtype=np.float64) * 2.0 ** -53
    above = 1.0 + np.arange(1, lim // 2 + 1, dtype=np.float64) * 2.0 ** -52
    for d in (below, above):
        assert np.all(np.abs(d - 1.0) <= 2.0 ** -30)
        want = 1.0 / np.sqrt(d)  # the reference: sqrt, then 1.0 / mag, both correctly rounded
        got = closed_form(d)
        bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
        assert bad.size == 0, (d[bad[:5]], got[bad[:5]], want[bad[:5]])


def test_inv_mag_near1_on_renormalised_vectors():
    # the re-normalisation v * r of unit vectors (as the specular's second norm() and the
    # reflection direction see them) matches the reference's norm bit for bit
    rng = np.random.default_rng(3)
    v = rng.normal(size=(3, 1 << 16))
    v = v * (1.0 / np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]))
    d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]
    assert np.all(np.abs(d - 1.0) <= 2.0 ** -30)
    want = v * (1.0 / np.sqrt(d))
    got = v * closed_form(d)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
