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
