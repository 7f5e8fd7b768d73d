"""Consensus parameters and the host-built tables the kernels consume.

The reference reads its parameters from module globals set in ``main``
(DuplexUMIConsensusReads.py:1432-1469) and evaluates, for every aligned entry,
``10 ** (-q / 10)`` and the post-UMI adjustment (:665-676), then for every
column ``int(round(-10 * math.log10(e'), 0))`` (:699-709).  The device must be
bit-exact with those Python/glibc results, so everything transcendental is
tabulated here on the host with the reference's own expressions:

* ``match[v] = 1 - p'(v)`` and ``mismatch[v] = p'(v) / 5`` for quality codes
  0..255 plus the '+' and '-' rows (the two factors of :594-600);
* ``post_threshold = 1 - 10 ** (-min_base_quality / 10)`` (:679-680);
* ``qthresh``: the exact double boundaries at which the consensus quality
  changes, found by bisection over the IEEE-754 ordering with ``math.log10``
  (so the device only compares doubles).
"""
from __future__ import annotations

import ctypes
import dataclasses
import math
import struct

LUT_PLUS, LUT_DEL, LUT_N = 256, 257, 258
MAX_QTHRESH = 257


@dataclasses.dataclass(frozen=True)
class ConsensusParams:
    """The numeric CLI flags of the reference (:10-91), same defaults."""
    min_map_quality: int = 20        # -q
    min_base_quality: int = 20
    min_reads: int = 1
    max_reads: int = 100
    max_base_quality: int = 60
    base_quality_shift: int = 0
    error_rate_post_labeling: int = 0
    error_rate_pre_labeling: int = 0
    deletion_score: int = 30
    no_insertion_score: int = 30

    @classmethod
    def from_args(cls, args):
        return cls(min_map_quality=args.min_map_quality, min_base_quality=args.min_base_quality,
                   min_reads=args.min_reads, max_reads=args.max_reads,
                   max_base_quality=args.max_base_quality,
                   base_quality_shift=args.base_quality_shift,
                   error_rate_post_labeling=args.error_rate_post_labeling,
                   error_rate_pre_labeling=args.error_rate_pre_labeling,
                   deletion_score=args.deletion_score, no_insertion_score=args.no_insertion_score)

    @classmethod
    def from_oracle_dict(cls, d):
        """Map the golden-fixture parameter names onto the CLI names."""
        return cls(min_base_quality=d["seqQ_threshold"], min_reads=d["min_reads"],
                   max_reads=d["max_reads"], max_base_quality=d["max_base_quality"],
                   base_quality_shift=d["base_quality_shift"], error_rate_post_labeling=d["post"],
                   error_rate_pre_labeling=d["pre"], deletion_score=d["deletion_score"],
                   no_insertion_score=d["no_insertion_score"])


def _post_adjust(ps: float, post: int) -> float:
    # :669 / :672 / :676, Python evaluation order
    return post * (1 - ps) + (1 - post) * ps + post * ps * 4 / 5


def error_probabilities(p: ConsensusParams):
    """p'(v) for v = 0..255, then '+' and '-' (:665-676)."""
    out = []
    for v in range(256):
        qa = min(v - p.base_quality_shift, p.max_base_quality)
        out.append(_post_adjust(10 ** (-qa / 10), p.error_rate_post_labeling))
    out.append(_post_adjust(10 ** (-p.no_insertion_score / 10), p.error_rate_post_labeling))
    out.append(_post_adjust(10 ** (-p.deletion_score / 10), p.error_rate_post_labeling))
    return out


def phred_raw(x: float) -> int:
    """``int(round(-10 * math.log10(x), 0))`` for finite x > 0 (:704)."""
    return int(round(-10 * math.log10(x), 0))


def _d2u(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _u2d(u: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", u))[0]


_MIN_POS = 1                       # bits of the smallest subnormal
_MAX_FIN = _d2u(1.7976931348623157e308)


def first_x_with_phred_at_most(k: int) -> float:
    """Smallest positive finite double x with phred_raw(x) <= k
    (phred_raw is non-increasing in x; bisection on the bit pattern)."""
    lo, hi = _MIN_POS, _MAX_FIN
    if phred_raw(_u2d(hi)) > k:
        return math.inf
    if phred_raw(_u2d(lo)) <= k:
        return _u2d(lo)
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if phred_raw(_u2d(mid)) <= k:
            hi = mid
        else:
            lo = mid
    return _u2d(hi)


def quality_thresholds(max_q: int):
    """qthresh[i] = first x with phred_raw(x) <= i - 1, i = 0..max_q."""
    return [first_x_with_phred_at_most(i - 1) for i in range(max_q + 1)]


def consensus_quality(x: float, max_q: int, qthresh) -> int:
    """Device rule (also used by tests to pin the table against :699-709)."""
    if not (x > 0):            # x <= 0 or NaN: the reference's ValueError branch
        return max_q
    c = sum(1 for t in qthresh if x >= t)
    return max_q - c


class DcrParams(ctypes.Structure):
    """Mirror of ``dcr_params`` (include/dcr.h)."""
    _fields_ = [("min_base_quality", ctypes.c_int32), ("max_base_quality", ctypes.c_int32),
                ("base_quality_shift", ctypes.c_int32), ("error_rate_post_labeling", ctypes.c_int32),
                ("error_rate_pre_labeling", ctypes.c_int32), ("deletion_score", ctypes.c_int32),
                ("no_insertion_score", ctypes.c_int32), ("n_qthresh", ctypes.c_int32),
                ("match", ctypes.c_double * LUT_N), ("mismatch", ctypes.c_double * LUT_N),
                ("post_threshold", ctypes.c_double),
                ("qthresh", ctypes.c_double * MAX_QTHRESH)]


_CACHE = {}


def build_dcr_params(p: ConsensusParams) -> DcrParams:
    if p in _CACHE:
        return _CACHE[p]
    if not (0 <= p.max_base_quality <= MAX_QTHRESH - 1):
        raise ValueError(f"--max_base_quality must be in [0, {MAX_QTHRESH - 1}]")
    s = DcrParams()
    s.min_base_quality = p.min_base_quality
    s.max_base_quality = p.max_base_quality
    s.base_quality_shift = p.base_quality_shift
    s.error_rate_post_labeling = p.error_rate_post_labeling
    s.error_rate_pre_labeling = p.error_rate_pre_labeling
    s.deletion_score = p.deletion_score
    s.no_insertion_score = p.no_insertion_score
    for i, pe in enumerate(error_probabilities(p)):
        s.match[i] = 1 - pe          # :598
        s.mismatch[i] = pe / 5       # :600 (len(likelihoods) - 1 == 5)
    s.post_threshold = 1 - 10 ** (-p.min_base_quality / 10)
    th = quality_thresholds(p.max_base_quality)
    s.n_qthresh = len(th)
    for i, t in enumerate(th):
        s.qthresh[i] = t
    _CACHE[p] = s
    return s
