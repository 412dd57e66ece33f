"""Integer identities the GPU kernels rely on, checked against the oracle restatement.

distance_d (DivergencePoint.cpp:53-65) against a mean histogram m_b = S_b / M truncates
(T)m_b and re-truncates the running magnitude after every bin.  Because frac(S_b/M) is 0
or lies in [1/M, 1-1/M], rounding never moves a value across an integer, so
  (T)m_b = floor(S_b/M) = F_b   and   mag = sum_b (p_b + F_b)
exactly (for M < ~1e11), i.e. distance_d(p, mean) = g(sum 2 min(p_b, F_b), mag_p + sum F_b):
a parallel integer reduction instead of a 4^k-long dependent floating-point chain.
"""
import numpy as np

import oracle_lib as O


def dd_identity(p, S, M):
    F = S // M
    dist = int(2 * np.minimum(p.astype(np.int64), F).sum())
    mag = int(p.astype(np.int64).sum() + F.sum())
    frac = dist / mag
    return np.fma(-frac, frac, 1.0) * 10000.0 if hasattr(np, "fma") else (1.0 - frac * frac) * 10000.0


def test_distance_d_identity_random():
    import math
    rng = np.random.default_rng(7)
    for t in range(3000):
        B = [16, 64, 256, 1024][t % 4]
        M = int(rng.integers(1, [5, 300, 200000][t % 3] + 1))
        maxv = int(rng.integers(1, 256))
        S = rng.integers(0, maxv + 1, size=B).astype(np.int64) * M + (rng.integers(0, M, size=B) if M > 1 else 0)
        S = np.minimum(S, maxv * M)
        p = rng.integers(0, maxv + 1, size=B).astype(np.uint8)
        mean = S.astype(np.float64) / float(M)
        want = O.distance_d(p, mean)
        F = S // M
        dist = int(2 * np.minimum(p.astype(np.int64), F).sum())
        mag = int(p.astype(np.int64).sum() + F.sum())
        frac = dist / mag
        got = math.fma(-frac, frac, 1.0) * 10000.0 if hasattr(math, "fma") else None
        if got is None:  # Python < 3.13: exact fma via fractions
            from fractions import Fraction
            got = float(Fraction(1) - Fraction(frac) * Fraction(frac)) * 10000.0
        assert got == want, (t, M, B)


def test_div32_float_reciprocal_division():
    """accum.hip's Div32: n / d for the worker count d (<= 256) and chunk indices n < 2^22 as
    trunc(float(n) * (1/d)) with one correction either way equals integer division, also when
    the float reciprocal is off by one ulp."""
    n = np.arange(0, 1 << 22, dtype=np.uint32)
    nf = n.astype(np.float32)
    for d in (1, 7, 8, 63, 127, 248, 255, 256):
        inv0 = np.float32(1.0) / np.float32(d)
        for inv in (inv0, np.nextafter(inv0, np.float32(0)), np.nextafter(inv0, np.float32(2))):
            q = (nf * inv).astype(np.uint32)
            r = n.astype(np.int64) - q.astype(np.int64) * d
            q = np.where(r < 0, q - 1, np.where(r >= d, q + 1, q))
            assert np.array_equal(q, n // d), d
