"""Exact arithmetic shortcuts the fast kernel relies on (dcr_kernels.hip),
proved exhaustively over their domains on the CPU."""
from fractions import Fraction


def _fma(a, b, c):
    """IEEE fused multiply-add: exact a * b + c, rounded once."""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def test_div1000_is_correctly_rounded():
    # div1000(k) = fma(fma(-q, 1000, k), 0.001, q), q = k * 0.001, for the
    # rounded means rint(1000 mean) in 0..1000 (:1015-1018)
    for k in range(1001):
        q = k * 0.001
        assert _fma(_fma(-q, 1000.0, float(k)), 0.001, q) == k / 1000, k


def test_uniform_depth_mean_rounding_margin():
    # a mean 1000 sum(e) / (d T) that is not a tie lies at least 1 / (2 d T)
    # from a half-integer: d <= 63, T <= 256 columns
    worst = min(Fraction(1, 2 * d * t) for d in (1, 63) for t in (1, 256))
    assert worst > Fraction(1, 10 ** 5)


def test_fast_rows_quotient_from_a_double_estimate():
    """k_fast_rows (dcr_kernels.hip): q = floor(25 S / (18018 T)) from a
    double estimate (num * (1 / den), each IEEE-rounded as on the device)
    fixed up by the integer remainder equals the exact integer quotient, over
    the whole domain's edges (S < 2^32, 1 <= T <= 240) and random values."""
    import numpy as np
    rng = np.random.default_rng(7)
    S = np.concatenate([rng.integers(0, 1 << 32, 200_000, dtype=np.int64),
                        np.array([0, 1, 720720, (1 << 32) - 1, (1 << 32) - 2], np.int64)])
    T = np.concatenate([rng.integers(1, 241, 200_000, dtype=np.int64), np.array([1, 1, 16, 240, 239], np.int64)])
    # exact multiples and their neighbours (remainder 0 / den - 1)
    k = rng.integers(0, 1 << 20, 50_000, dtype=np.int64)
    Tm = rng.integers(1, 241, 50_000, dtype=np.int64)
    for dlt in (-1, 0, 1):
        Sm = (k * 18018 * Tm + dlt) // 25
        ok = (Sm >= 0) & (Sm < (1 << 32))
        S = np.concatenate([S, Sm[ok]])
        T = np.concatenate([T, Tm[ok]])
    num = 25 * S
    den = 18018 * T
    q = (num.astype(np.float64) * (1.0 / den.astype(np.float64))).astype(np.int64)
    r = num - q * den
    q = np.where(r < 0, q - 1, q)
    r = np.where(r < 0, r + den, r)
    q = np.where(r >= den, q + 1, q)
    assert np.array_equal(q, num // den)
