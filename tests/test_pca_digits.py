"""The int8 digit scheme of the exact PCA engine (kernels/pca_ozaki.hip), emulated in numpy:
digit ranges, representation error, the int32 headroom of a flush, and the a priori bound on
one product that pca.cpp reports (summed over rows) — checked against exact rational arithmetic.
CPU only: the GPU tests compare the kernel itself against np.cov (tests/test_pca_gpu.py)."""
from fractions import Fraction

import numpy as np

DIGITS = 7


def digits(v, E):
    """The kernel's digit loop: w = v 2^(6 - E), t_0 = rint(w), then 6 x (w *= 128, rint)."""
    w = np.ldexp(v, 6 - E)
    out = []
    t = np.rint(w)
    out.append(t)
    w = w - t
    for _ in range(1, DIGITS):
        w = w * 128.0
        t = np.rint(w)
        out.append(t)
        w = w - t
    return np.stack(out).astype(np.int64), w  # (residual in units of 2^(E - 48))


def exponent(m):
    return 0 if m == 0 else int(np.frexp(m)[1])  # m < 2^E (frexp: m = f 2^e, 0.5 <= f < 1)


def test_digits_in_int8_range_and_reconstruct():
    rng = np.random.default_rng(0)
    x = (rng.normal(size=20000) * rng.uniform(0.01, 100, size=20000)).astype(np.float32)
    s = np.float64(np.float32(x[:256].mean()))
    v = x.astype(np.float64) - s
    E = exponent(np.abs(v).max())
    t, _ = digits(v, E)
    assert t.min() >= -64 and t.max() <= 64
    # v = 2^(E-6) sum_p t_p 2^(-7p) + rho, |rho| <= 2^(E-49)
    for i in range(0, 20000, 997):
        approx = sum(Fraction(int(t[p, i])) / 2 ** (7 * p) for p in range(DIGITS)) * \
            Fraction(2) ** (E - 6)
        assert abs(Fraction(float(v[i])) - approx) <= Fraction(2) ** (E - 49)


def test_level_sums_fit_int32_for_a_flush():
    # |t_p t_q| <= 2^12, <= 7 products per level and row, 32 rows a block, 2048 blocks a flush
    assert 7 * 2 ** 12 * 32 * 2048 < 2 ** 31


def test_product_error_within_the_reported_bound():
    """Per row and entry:
    |v_j v_k - sum_{p+q<=6} t_p u_q 2^(E_j+E_k-12-7(p+q))| <= 8.04 2^(E_j+E_k-49)."""
    rng = np.random.default_rng(1)
    a = rng.normal(size=3000) * 3.0
    b = rng.normal(size=3000) * 0.02 + 0.5
    Ea, Eb = exponent(np.abs(a).max()), exponent(np.abs(b).max())
    ta, _ = digits(a, Ea)
    tb, _ = digits(b, Eb)
    worst = Fraction(0)
    for i in range(0, 3000, 37):
        s = Fraction(0)
        for p in range(DIGITS):
            for q in range(DIGITS - p):
                s += Fraction(int(ta[p, i]) * int(tb[q, i])) / 2 ** (7 * (p + q))
        s *= Fraction(2) ** (Ea + Eb - 12)
        err = abs(Fraction(float(a[i])) * Fraction(float(b[i])) - s)
        worst = max(worst, err / Fraction(2) ** (Ea + Eb - 49))
    assert worst <= Fraction(804, 100)
