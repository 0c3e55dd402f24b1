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

// ---------------------------------------------------------------- correctly rounded acos / sin
// For the sphere UV's texel-boundary path only (rt_device.h sphere_texel_uv): a texel coordinate within
// rounding of an integer decides the texel by the last bit of acos / sin, where rt_acos and ocml's sin may
// differ from glibc's by an ulp.  These evaluate in double-double (error-free transforms on FMA, Taylor
// coefficients as double-double constants) to ~2^-100 relative and round once, so they return the
// correctly rounded result except for values within ~2^-100 of a rounding midpoint; glibc 2.35's acos /
// sin are themselves correctly rounded on all but ~0.05 % / ~0.14 % of inputs (measured against
// libquadmath, tests/test_rt_math.py).  Slow (hundreds of flops) and only ever taken by the rare lanes
// that need them.
struct rt_dd { double hi, lo; };
RT_HD static inline rt_dd rt_two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
RT_HD static inline rt_dd rt_fast_two_sum(double a, double b) {      // |a| >= |b| (or a == 0)
  const double s = a + b;
  return {s, b - (s - a)};
}
RT_HD static inline rt_dd rt_dd_add(rt_dd a, rt_dd b) {
  rt_dd s = rt_two_sum(a.hi, b.hi);
  const rt_dd t = rt_two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = rt_fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return rt_fast_two_sum(s.hi, s.lo);
}
RT_HD static inline rt_dd rt_dd_mul(rt_dd a, rt_dd b) {
  const double p = a.hi * b.hi;
  double e = fma(a.hi, b.hi, -p);
  e += a.hi * b.lo + a.lo * b.hi;
  return rt_fast_two_sum(p, e);
}
// sin(t) and cos(t) for a double-double |t| <= pi/4: Taylor to t^23 / t^24 (next terms < 2^-92 relative)
RT_HD static inline rt_dd rt_sin_poly_dd(rt_dd t) {
  const double c[11][2] = {
      {-0x1.5555555555555p-3, -0x1.5555555555555p-57}, {0x1.1111111111111p-7, 0x1.1111111111111p-63},
      {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73}, {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},
      {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80}, {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},
      {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97}, {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},
      {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112}, {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},
      {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130}};            // (-1)^k / (2k+1)!, k = 1..11
  const rt_dd u = rt_dd_mul(t, t);
  rt_dd acc = {c[10][0], c[10][1]};
#pragma unroll
  for (int k = 9; k >= 0; --k) acc = rt_dd_add(rt_dd_mul(acc, u), rt_dd{c[k][0], c[k][1]});
  return rt_dd_add(t, rt_dd_mul(t, rt_dd_mul(u, acc)));
}
RT_HD static inline rt_dd rt_cos_poly_dd(rt_dd t) {
  const double c[12][2] = {
      {-0x1.0000000000000p-1, 0.0}, {0x1.5555555555555p-5, 0x1.5555555555555p-59},
      {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65}, {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},
      {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76}, {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},
      {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92}, {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},
      {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107}, {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},
      {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124}, {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135}};   // (-1)^k / (2k)!
  const rt_dd u = rt_dd_mul(t, t);
  rt_dd acc = {c[11][0], c[11][1]};
#pragma unroll
  for (int k = 10; k >= 0; --k) acc = rt_dd_add(rt_dd_mul(acc, u), rt_dd{c[k][0], c[k][1]});
  return rt_dd_add(rt_dd{1.0, 0.0}, rt_dd_mul(u, acc));
}
// asin(t) for a double-double |t| <= 1/2: fdlibm's asin (about an ulp) as the start, one Newton step on
// sin in double-double (the start's error squared is ~2^-106; the correction itself needs only double).
RT_HD static inline rt_dd rt_asin_dd(rt_dd t) {
  const double a0 = t.hi + t.hi * rt_asin_r(t.hi * t.hi);
  const rt_dd f = rt_dd_add(rt_sin_poly_dd(rt_dd{a0, 0.0}), rt_dd{-t.hi, -t.lo});     // sin(a0) - t
  return rt_fast_two_sum(a0, -f.hi / cos(a0));
}
RT_HD static inline double rt_acos_cr(double x) {
  const rt_dd pi = {0x1.921fb54442d18p+1, 0x1.1a62633145c07p-53}, pio2 = {0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54};
  const double ax = fabs(x);
  if (!(ax < 1.0)) return rt_acos(x);                  // +-1 (exact), |x| > 1 and NaN (NaN)
  if (ax <= 0.5) {                                     // pi/2 - asin(x)
    const rt_dd r = rt_dd_add(pio2, rt_asin_dd(rt_dd{-x, 0.0}));
    return r.hi + r.lo;
  }
  const double z = (1.0 - ax) * 0.5;                   // exact (Sterbenz)
  const double s = sqrt(z);
  const rt_dd sd = rt_fast_two_sum(s, fma(-s, s, z) / (s + s));     // sqrt(z) to ~2^-106
  const rt_dd a = rt_asin_dd(sd);
  const rt_dd a2 = {2.0 * a.hi, 2.0 * a.lo};            // 2 asin(sqrt z), exact scaling
  if (x > 0.0) return a2.hi + a2.lo;
  const rt_dd r = rt_dd_add(pi, rt_dd{-a2.hi, -a2.lo}); // pi - 2 asin(sqrt z)
  return r.hi + r.lo;
}
// sin(x) for x in [0, pi] (the sphere UV's phi = acos(...)); other x: the platform's sin.  pi/2 - x and
// pi - x are exact (Sterbenz) on their branches; pi is carried as a double-double.
RT_HD static inline double rt_sin_cr(double x) {
  const double pio2_hi = 0x1.921fb54442d18p+0, pio2_lo = 0x1.1a62633145c07p-54;
  const double pi_hi = 0x1.921fb54442d18p+1, pi_lo = 0x1.1a62633145c07p-53;
  if (!(x >= 0.0 && x <= pi_hi)) return sin(x);
  rt_dd r;
  if (x <= 0x1.921fb54442d18p-1) r = rt_sin_poly_dd(rt_dd{x, 0.0});                          // x <= pi/4
  else if (x <= 0x1.2d97c7f3321d2p+1) r = rt_cos_poly_dd(rt_fast_two_sum(pio2_hi - x, pio2_lo));   // <= 3pi/4
  else r = rt_sin_poly_dd(rt_fast_two_sum(pi_hi - x, pi_lo));
  return r.hi + r.lo;
}
