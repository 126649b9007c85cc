"""Restated numpy 2.x float32 ``np.sin``/``np.cos`` -- TEST ORACLE ONLY.

The reference computes every direction vector as
``np.stack((np.sin(b, dtype=np.float32), np.cos(b, dtype=np.float32)), -1)``
(astro/util.py:87-92).  numpy 2.2.6 evaluates float32 sin/cos on x86 with a
vectorised algorithm (numpy/_core/src/umath/loops_trigonometric.dispatch.cpp,
a third-party dependency of the reference; pinned version in configs.json):

  q  = rint(x * 2/pi) = fma(x, 2/pi, 1.5*2**23) - 1.5*2**23
  r  = x - q*pi/2 as three FMAs (Cody-Waite, pi/2 split hi/med/lo)
  sin(r) ~ r + r^3*P(r^2), cos(r) ~ Q(r^2)  (minimax, Horner with FMAs)
  quadrant select/negate from int(q) (+1 for cos)
  |x| > 117435.992 (sin) / 71476.0625 (cos): scalar libm fallback

It is NOT correctly rounded (about 15% of inputs differ by 1 ulp from the
rounded float64 result), so a bit-exact kernel must run this exact algorithm.
This module restates it with an exact float32 FMA (float64 product + round-
to-odd sum, then one rounding to float32) and tests/test_oracle_golden.py
checks it bit for bit against ``np.sin``/``np.cos`` on millions of inputs.
The HIP kernel (astro_amd/csrc/astro_kernels.hip, ``np_sincosf``) runs the
same sequence with hardware ``v_fma_f32``.
"""
import numpy as np

F = np.float32


def _hx(s):
    return F(float.fromhex(s))


TWO_OVER_PI = _hx('0x1.45f306p-1')
PIO2_HI = _hx('-0x1.921fb0p+00')
PIO2_MED = _hx('-0x1.5110b4p-22')
PIO2_LO = _hx('-0x1.846988p-48')
RINT_MAGIC = _hx('0x1.800000p+23')
COS_C = [_hx('0x1.98e616p-16'), _hx('-0x1.6c06dcp-10'), _hx('0x1.55553cp-5'),
         _hx('-0x1.000000p-1'), _hx('0x1.000000p+0')]
SIN_C = [_hx('0x1.7d3bbcp-19'), _hx('-0x1.a06bbap-13'), _hx('0x1.11119ap-07'),
         _hx('-0x1.555556p-03')]
MAX_CODY_SIN = F(117435.992)
MAX_CODY_COS = F(71476.0625)


def fma32(a, b, c):
    """Correctly rounded float32 a*b+c (numpy arrays of float32)."""
    a = np.asarray(a, np.float32).astype(np.float64)
    b = np.asarray(b, np.float32).astype(np.float64)
    c = np.asarray(c, np.float32).astype(np.float64)
    p = a * b                      # exact: 24+24 bits <= 53
    s = p + c
    bb = s - p
    e = (p - (s - bb)) + (c - bb)  # TwoSum: p + c == s + e exactly
    even = (s.view(np.int64) & 1) == 0
    fix = (e != 0) & even
    toward = np.where(e > 0, np.inf, -np.inf)
    s = np.where(fix, np.nextafter(s, toward), s)   # round-to-odd at 53 bits
    return s.astype(np.float32)


def _sincos(x, want_cos):
    x = np.asarray(x, dtype=np.float32)
    q = fma32(x, TWO_OVER_PI, RINT_MAGIC) - RINT_MAGIC
    r = fma32(q, PIO2_HI, x)
    r = fma32(q, PIO2_MED, r)
    r = fma32(q, PIO2_LO, r)
    r2 = r * r
    c = fma32(COS_C[0], r2, COS_C[1])
    for k in COS_C[2:]:
        c = fma32(c, r2, k)
    s = fma32(SIN_C[0], r2, SIN_C[1])
    for k in SIN_C[2:]:
        s = fma32(s, r2, k)
    s = fma32(s, r2, F(0))
    s = fma32(s, r, r)
    iq = q.astype(np.int32) + (1 if want_cos else 0)
    out = np.where((iq & 1) == 0, s, c)
    out = np.where((iq & 2) == 2, F(0) - out, out)
    lim = MAX_CODY_COS if want_cos else MAX_CODY_SIN
    return out.astype(np.float32), np.abs(x) <= lim


def sin32(x):
    """numpy-exact float32 sin for |x| <= 117435.992 (NaN outside)."""
    v, ok = _sincos(x, False)
    return np.where(ok, v, np.float32(np.nan))


def cos32(x):
    """numpy-exact float32 cos for |x| <= 71476.0625 (NaN outside)."""
    v, ok = _sincos(x, True)
    return np.where(ok, v, np.float32(np.nan))
