// rt_math.h -- acos for the render kernels (host + device).
//
// Why not ocml's acos: it needs 32 VGPRs and ~100 VALU instructions per call, and the shading
// code calls it per light per hit -- it set the kernel's register peak.  This one follows the
// classic fdlibm e_acos.c decomposition (rational minimax P/Q for asin on |x| < 1/2, half-angle
// forms outside; published, freely distributable coefficients), then finishes each branch with
// error-free transforms (Fast2Sum / an FMA-exact square-root residual) so the final rounding is
// the only significant one: measured against glibc (the reference's libm) it differs on ~0.1% of
// inputs by 1 ulp (tests/test_rt_math.py; ocml: 6.5%, plain fdlibm: 5.1%).
// fma() here is an explicit, deterministic part of THIS function -- the reference's own
// arithmetic is still evaluated without contraction everywhere else.
#pragma once
#ifndef __HIPCC_RTC__
#include <math.h>
#endif

#ifndef RT_HD
#define RT_HD
#endif

// Operations whose operand ranges rt_acos guarantees (|x| < 1 branches): sqrt of z in
// (2^-54, 1/4], p / q with p in (2^-120, 1) and q in [1/2, 1], and the residual quotient
// fma(-s,s,z) / 2s (numerator 0 or |.| >= 2^-160).  The device build substitutes cores without the
// scaling steps that are identities on those ranges (rt_device.h: bit-identical results).
#ifndef RT_SQRT_IN_RANGE
#define RT_SQRT_IN_RANGE(x) sqrt(x)
#endif
#ifndef RT_DIV_IN_RANGE
#define RT_DIV_IN_RANGE(a, b) ((a) / (b))
#endif

RT_HD static inline double rt_asin_r(double z) {       // R(z) = P(z) / Q(z), asin(x) = x + x*R(x^2)
  const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
               pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
               pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
               qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
               qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
  double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  return RT_DIV_IN_RANGE(p, q);
}

RT_HD static inline double rt_acos(double x) {
  const double pi_hi = 3.14159265358979311600e+00, pi_lo = 1.22464679914735317720e-16;
  const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
  const double ax = fabs(x);
  if (!(ax < 1.0)) {
    if (x == 1.0) return 0.0;
    if (x == -1.0) return pi_hi + pi_lo;
    return (x - x) / (x - x);                          // |x| > 1 or NaN -> NaN
  }
  if (ax < 0.5) {                                      // pi/2 - (x + x R(x^2))
    if (ax <= 0x1p-57) return pio2_hi + pio2_lo;
    const double t = x * rt_asin_r(x * x);
    const double s = pio2_hi - x;                      // Fast2Sum: |pio2_hi| > |x|
    const double e = (pio2_hi - s) - x;
    return s + ((e + pio2_lo) - t);
  }
  const double z = (ax == x ? 1.0 - x : 1.0 + x) * 0.5;   // exact (Sterbenz)
  const double s = RT_SQRT_IN_RANGE(z);
  const double sl = RT_DIV_IN_RANGE(fma(-s, s, z), s + s);           // sqrt(z) = s + sl to ~2^-106
  const double r = rt_asin_r(z);
  if (x > 0.0) {                                       // 2 asin(sqrt z)
    return 2.0 * (s + (sl + s * r));
  }
  const double h = 2.0 * s;                            // pi - 2 asin(sqrt z)
  const double a = pi_hi - h;                          // Fast2Sum: pi_hi > h
  const double e = (pi_hi - a) - h;
  return a + ((e + pi_lo) - 2.0 * (sl + s * r));
}
