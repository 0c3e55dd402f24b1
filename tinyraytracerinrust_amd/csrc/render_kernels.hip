// render_kernels.hip -- gfx950 (MI355X, CDNA4) kernels for the TinyRaytracer render path, and
// the device-context half of the C ABI (rt_ctx_*, rt_render_*).
//
// One thread per pixel; each 64-lane wave owns an 8x8 pixel tile (coherent primary rays,
// fewer divergent CSG/shade branches than a 64x1 row strip); a 256-thread workgroup is a 16x16
// tile.  All arithmetic is IEEE f64 with NO contraction (Rust never fuses): the file is
// compiled with -ffp-contract=off and the pragma below.  sqrt and division lower to correctly
// rounded sequences on gfx950 (verified bit-exact against glibc, profiles/r01_libm_probe.txt);
// acos is rt_acos (rt_math.h: 1 ulp from glibc on ~0.4% of inputs, and far fewer registers than
// ocml's); sin comes from ocml and may differ from glibc by 1 ulp (DESIGN.md "Parity").
//
// The reference's recursion (get_ray_color calling itself for refraction and reflection,
// raytracer.rs:242-280) becomes an explicit per-lane frame stack combined in the same
// post-order: child colour C folds into its parent as in_range(A + in_range(C * w)) where
// A = parent.intensify(1 - w) -- exactly the `final.intensify(1-w) + R.intensify(w)` of
// raytracer.rs:256-257 / :278-279.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdlib.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>
#include <vector>

#define RT_HD __device__
#include "rt_blob.h"
// Correctly rounded sqrt(x) and 1/sqrt-derived reciprocals without their range handling.
// For f64 `sqrt` and `/` the compiler emits (gfx950) scaled Newton sequences:
//   sqrt(x): x scaled by 2^256 if x < 2^-767, y = rsq(x), g = x*y, h = 0.5*y, r = fma(-h,g,0.5),
//            g = fma(g,r,g), h = fma(h,r,h), twice {d = fma(-g,g,x), g = fma(d,h,g)}, g scaled back,
//            and x itself returned for +-0 / +inf (17 VALU instructions);
//   a / b:   v_div_scale of b and of a, rcp, 4 Newton fmas, mul, fma, v_div_fmas, v_div_fixup (11).
// For x in [2^-767, DBL_MAX] the scalings are by 2^0 and the class select returns g, so the
// unscaled core below is the SAME operation sequence on the same values: bit-identical.  Then
// l = sqrt(x) is in [2^-383.5, 2^512): for 1.0 / l v_div_scale scales neither operand (both
// normal, exponent gap < 768, 1/l and the quotient normal), so v_div_fmas is a plain fma (VCC 0),
// the mul by the numerator 1.0 is exact, and v_div_fixup returns its positive normal operand:
// again the same values.  The range test is wave-uniform (one ballot), outside it the compiler's
// sequences run.  RT_FAST_SQRT=0 restores the plain `sqrt` / `/` everywhere.
#ifndef RT_FAST_SQRT
#define RT_FAST_SQRT 1
#endif
static __device__ __forceinline__ double sqrt_core(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
static __device__ __forceinline__ double recip_core(double l) {     // 1.0 / l for l in [2^-384, 2^512]
  const double nl = -l;
  const double r = __builtin_amdgcn_rcp(l);
  const double f0 = __builtin_fma(nl, r, 1.0);
  const double f1 = __builtin_fma(r, f0, r);
  const double f2 = __builtin_fma(nl, f1, 1.0);
  const double f3 = __builtin_fma(f1, f2, f1);
  const double f4 = __builtin_fma(nl, f3, 1.0);            // mul = 1.0 * f3 = f3
  return __builtin_fma(f4, f3, f3);
}
// a / b when neither v_div_scale scales (both operands normal, exponent gap < 768, quotient
// normal, |a| >= 2^-969) or a == 0: the compiler's sequence with those identities dropped;
// v_div_fixup is kept, so a zero numerator gives the same signed zero.
static __device__ __forceinline__ double div_core(double a, double b) {
  const double nb = -b;
  const double r = __builtin_amdgcn_rcp(b);
  const double f0 = __builtin_fma(nb, r, 1.0);
  const double f1 = __builtin_fma(r, f0, r);
  const double f2 = __builtin_fma(nb, f1, 1.0);
  const double f3 = __builtin_fma(f1, f2, f1);
  const double m = a * f3;
  const double f4 = __builtin_fma(nb, m, a);
  return __builtin_amdgcn_div_fixup(__builtin_fma(f4, f3, m), b, a);
}
// rt_math.h's rt_acos takes these for the operations whose operand ranges it guarantees.
#ifndef RT_ACOS_CORES
#define RT_ACOS_CORES 1
#endif
#if RT_FAST_SQRT && RT_ACOS_CORES
#define RT_SQRT_IN_RANGE(x) sqrt_core(x)
#define RT_DIV_IN_RANGE(a, b) div_core(a, b)
#endif
#include "rt_math.h"
#include "scene.h"

#ifdef RT_ABLATE_FAST_ACOS   // diagnostic cost-split builds only (wrong colours): acos in f32
#define rt_acos(x) ((double)acosf((float)(x)))
#endif

#pragma clang fp contract(off)

// Diagnostic section-cycle build (make profile-sections; never the product): wave-cycles spent
// in each part of trace(), summed over all waves with one atomic per wave per section entry.
#ifdef RT_PROF
__device__ unsigned long long g_rt_prof[8];
#define PROF_T0(v) const long long v = clock64()
#define PROF_ADD(sec, v)                                                              \
  do {                                                                                \
    const long long d_ = clock64() - (v);                                             \
    if ((int)__lane_id() == __ffsll((long long)__ballot(1)) - 1)                       \
      atomicAdd(&g_rt_prof[sec], (unsigned long long)d_);                             \
  } while (0)
#else
#define PROF_T0(v) (void)0
#define PROF_ADD(sec, v) (void)0
#endif

// Diagnostic event-count build (make diag NAME=cnt DIAG=-DRT_COUNT; never the product): per ray
// category (0 primary, 1 secondary, 2 shadow) rays, object box tests, objects entered, leaf box
// tests, leaf evaluations (all / sphere / plane / cube), CSG filter calls; lane-events, one atomic
// per wave per event.
#ifdef RT_COUNT
__device__ unsigned long long g_rt_cnt[64];
#define CNT(i)                                                                          \
  do {                                                                                  \
    const unsigned long long m_ = __ballot(1);                                          \
    if ((int)__lane_id() == __ffsll((long long)m_) - 1) atomicAdd(&g_rt_cnt[i], (unsigned long long)__popcll(m_)); \
  } while (0)
#define CNTW(i)                                                                         \
  do {                                                                                  \
    const unsigned long long m_ = __ballot(1);                                          \
    if ((int)__lane_id() == __ffsll((long long)m_) - 1) atomicAdd(&g_rt_cnt[i], 1ull); \
  } while (0)
#else
#define CNT(i) (void)0
#define CNTW(i) (void)0
#endif

namespace {

// Scene tables are read-only for the whole launch: view them through the CONSTANT address space
// (4) so uniform-index reads compile to scalar (SMEM) loads instead of per-lane VMEM loads.
#ifdef RT_DIAG_LDS_SCENE                 // diagnostic A/B build only (make diag): scene tables staged in LDS
#define CAS __attribute__((address_space(3)))
#else
#define CAS __attribute__((address_space(4)))
#endif
template <class T> using cptr = const CAS T*;
template <class T> __device__ __forceinline__ cptr<T> as_const(const T* p) { return (cptr<T>)p; }

struct DS {                         // device view of RtDevScene
  cptr<RtObject> objects;
  cptr<RtTrav> trav;
  cptr<RtTrav> strav;               // shadow-ray walk of scenes without a transparent object
  cptr<RtNode> nodes;
  cptr<RtLeaf> leaves;
  cptr<RtProg> prog;
  cptr<RtLight> lights;
  cptr<RtTexture> textures;
  const uint8_t* texels;            // per-lane texel gathers stay global (vector) loads
  int n_objects, n_lights, n_trav, n_strav;
  int shadow_early_out;
};

constexpr double EPS = RT_EPSILON;
#ifndef RT_PLANE_AXIS
#define RT_PLANE_AXIS 1             // axis-aligned planes: one product per dot in the traversals
#endif
#ifndef RT_NEAREST_ORDER
#define RT_NEAREST_ORDER 1          // reflection-only kernels: nearest-hit walk in the shadow walk's order (tie-exact)
#endif
#ifndef RT_SHADOW_ORDER
#define RT_SHADOW_ORDER 1           // reflection-only kernels: shadow rays walk the likeliest occluders first
#endif
#ifndef RT_CONST_FILTER
#define RT_CONST_FILTER 1           // skip hit filters the host proved constant (RtLeaf::filter_const) in the
                                    // refraction kernels (SHARE): spinning_globes' glass shells, 10.5 % faster;
                                    // in the reflection-only megakernel the test cost 4 more spilled VGPRs
                                    // (profiles/r02co_const_filter_ab.txt)
#endif
#ifndef RT_SPHERE_SHARE
#define RT_SPHERE_SHARE 1           // concentric sphere leaves with one transform share their ray terms
#endif
#ifndef RT_SPHERE_SHARE_CHAIN
#define RT_SPHERE_SHARE_CHAIN 1     // the refraction-chain kernel shares sphere terms too
#endif
constexpr double PI_D = 3.14159265358979323846;   // std::f64::consts::PI

struct V3 { double x, y, z; };
struct Col { double r, g, b; };

__device__ __forceinline__ V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 scale(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ bool wave_sqrt_core_ok(double x) {
  return __ballot(!(x >= 0x1p-767 && x <= 0x1.fffffffffffffp+1023)) == 0;
}
__device__ __forceinline__ double sqrt_rt(double x) {
#if RT_FAST_SQRT
  if (wave_sqrt_core_ok(x)) return sqrt_core(x);
#endif
  return sqrt(x);
}
__device__ __forceinline__ double len(V3 a) { return sqrt_rt(dot(a, a)); }
// l = len(a) and il = 1.0 / l, as `len(a)` and `1.0 / len(a)` compute them
__device__ __forceinline__ void len_inv(V3 a, double* l, double* il) {
  const double x = dot(a, a);
#if RT_FAST_SQRT
  if (wave_sqrt_core_ok(x)) {
    *l = sqrt_core(x);
    *il = recip_core(*l);
    return;
  }
#endif
  *l = sqrt(x);
  *il = 1.0 / *l;
}
__device__ __forceinline__ V3 normalized(V3 a) {
  double l, il;
  len_inv(a, &l, &il);
  return scale(a, il);
}
template <class P> __device__ __forceinline__ V3 ld3(P p) { return {p[0], p[1], p[2]}; }
// transform_vector (transformation.rs:53-59) with rows m[0..3], m[4..7], m[8..11]
template <class P> __device__ __forceinline__ V3 xf(P m, V3 v) {
  return {m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3],
          m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7],
          m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11]};
}
// transform_vector by a diagonal-affine matrix (RtLeaf::xdiag): bit-identical to xf() for finite
// inputs (rt_blob.h), 6 flops instead of 18.
template <class P> __device__ __forceinline__ V3 xf_diag(P m, V3 v) {
  return {m[0] * v.x + m[3], m[5] * v.y + m[7], m[10] * v.z + m[11]};
}
__device__ __forceinline__ bool finite3(V3 v) { return isfinite(v.x) && isfinite(v.y) && isfinite(v.z); }
// Is every active lane's vector finite?  Wave-uniform, so the short transform is a scalar branch.
__device__ __forceinline__ bool wave_finite(V3 a) { return __ballot(!finite3(a)) == 0; }
__device__ __forceinline__ bool wave_finite(V3 a, V3 b) { return __ballot(!(finite3(a) && finite3(b))) == 0; }
// The leaf's inverse transform of a point (transformation.rs:53-59); `fin` = wave_finite(v).
__device__ __forceinline__ V3 leaf_inv_xf(cptr<RtLeaf> L, V3 v, bool fin) {
  if (L->xdiag == RT_XF_IDENTITY && fin) return v;
  if (L->xdiag && fin) return xf_diag(L->inv, v);
  return xf(L->inv, v);
}

// color.rs:36-53: clamp each channel (NaN passes through)
// FC (fast clamp): the same clamp as two min/max instructions instead of two compares and four
// selects.  fmin(fmax(x, 0), 1) equals `x < 0 ? 0 : (x > 1 ? 1 : x)` bit for bit for every x
// except NaN (maxNum drops it) and -0 (max(-0, +0) is +0).  The host sets RtDevScene::colour_fast
// only when no colour-op operand can be NaN, negative or -0 (every material / light colour channel
// finite and >= +0, every reflectivity and transparency finite in [0, 1]: then every factor of
// every colour op is finite and >= +0, see rt::flatten), and the kernels take FC = true only then.
// 3.4 % faster on 4K globes, 2 % on spinning_globes (profiles/r02ab.txt).
template <bool FC = false> __device__ __forceinline__ double in_limit(double x) {
  if constexpr (FC) return __builtin_fmin(__builtin_fmax(x, 0.0), 1.0);
  else return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);
}
template <bool FC = false> __device__ __forceinline__ Col in_range(double r, double g, double b) {
  return {in_limit<FC>(r), in_limit<FC>(g), in_limit<FC>(b)};
}
template <bool FC = false> __device__ __forceinline__ Col intensify(Col c, double k) { return in_range<FC>(c.r * k, c.g * k, c.b * k); }
template <bool FC = false> __device__ __forceinline__ Col cmul(Col a, Col b) { return in_range<FC>(a.r * b.r, a.g * b.g, a.b * b.b); }
template <bool FC = false> __device__ __forceinline__ Col cadd(Col a, Col b) { return in_range<FC>(a.r + b.r, a.g + b.g, a.b + b.b); }
// `(c * 255.0) as u8` (easy_pixbuf.rs:49-52): saturating truncation, NaN -> 0
__device__ __forceinline__ uint32_t to_u8(double c) {
  double v = c * 255.0;
  if (!(v > 0.0)) return 0u;
  if (v >= 255.0) return 255u;
  return (uint32_t)v;
}

// ------------------------------------------------------------------ primitives (math_shapes.rs)
template <class P> __device__ __forceinline__ bool on_plane(P pl, V3 q) {        // :162-164
  return fabs(pl[0] * q.x + pl[1] * q.y + pl[2] * q.z + pl[3]) < EPS;
}

__device__ bool leaf_inside(cptr<RtLeaf> L, V3 p, bool fin) {
  int k = L->kind;
  if (k == RT_N_PLANE) return false;                                        // :186-188
  V3 q = leaf_inv_xf(L, p, fin);
  if (k == RT_N_SPHERE) return len(sub(q, ld3(L->c))) <= L->r_eps;         // :70-74
  return q.x <= L->hi[0] && q.x >= L->lo[0] && q.y <= L->hi[1] &&          // :319-328
         q.y >= L->lo[1] && q.z <= L->hi[2] && q.z >= L->lo[2];
}

__device__ bool leaf_on_surface(cptr<RtLeaf> L, V3 p, bool fin) {
  V3 q = leaf_inv_xf(L, p, fin);
  int k = L->kind;
  if (k == RT_N_SPHERE) return fabs(len(sub(q, ld3(L->c))) - L->radius) < EPS;   // :76-80
  if (k == RT_N_PLANE) return on_plane(L->pl[0], q);                            // :190-194
  bool bx = L->lo_e[0] <= q.x && q.x <= L->hi_e[0];                              // :330-355
  bool by = L->lo_e[1] <= q.y && q.y <= L->hi_e[1];
  bool bz = L->lo_e[2] <= q.z && q.z <= L->hi_e[2];
  if (by && bx && (on_plane(L->pl[0], q) || on_plane(L->pl[5], q))) return true;
  if (bz && bx && (on_plane(L->pl[1], q) || on_plane(L->pl[4], q))) return true;
  if (by && bz && (on_plane(L->pl[2], q) || on_plane(L->pl[3], q))) return true;
  return false;
}

__device__ V3 leaf_normal(cptr<RtLeaf> L, V3 p, bool fin) {
  int k = L->kind;
  if (k == RT_N_PLANE) return ld3(L->pn[0]);                               // :182-184
  V3 q = leaf_inv_xf(L, p, fin);
  if (k == RT_N_SPHERE) {                                                  // :64-68
    V3 n = sub(q, ld3(L->c));
    return normalized(sub(xf(L->mat, n), ld3(L->mat_o)));
  }
  for (int i = 0; i < 6; ++i)                                              // :292-317
    if (on_plane(L->pl[i], q)) return ld3(L->pn[i]);
  return {1.0, 1.0, 1.0};
}

// MathSphere::get_uv_coordinates (:82-114): the centre is subtracted BEFORE the inverse transform
__device__ void sphere_uv(cptr<RtLeaf> L, V3 p, double* u, double* v) {
#ifdef RT_ABLATE_NO_UV       // diagnostic cost-split builds only (wrong colours)
  *u = *v = 0.0;
  if (p.x > 1e300) return;
#endif
  V3 q = xf(L->inv, sub(p, ld3(L->c)));           // per shaded hit only: no short form
  q = scale(normalized(q), 1.0 - EPS);
  double phi = rt_acos(-((0.0 * q.x + 1.0 * q.y) + 0.0 * q.z));             // up = (0,1,0)
  if (isnan(phi)) phi = 0.0;
  double theta = (rt_acos(((q.x * 0.0 + q.y * 0.0) + q.z * -1.0) / sin(phi))) / (2.0 * PI_D);   // u_zero = (0,0,-1)
  if (isnan(theta)) theta = 0.0;
  *v = phi / PI_D;
  *u = ((-1.0 * q.x + 0.0 * q.y) + 0.0 * q.z > 0.0) ? 1.0 - theta : theta;  // u_qrtr = (-1,0,0)
}

// Candidate hit distances of one primitive for the world ray (ro, rd):
// RTObject::intersects (rt_object.rs:28-31) = reverse_transform_ray + MathShape::intersects.
// `fin` = wave_finite(ro, rd): selects the exact short forms for identity / diagonal-affine
// leaves (rt_blob.h).  POS: the caller accepts only t > EPS (the traversals), so a plane whose
// distance is provably <= 0 from the signs alone skips its division (see the plane branch).
// SphereShare: a traversal's per-lane record of the last sphere leaf's ray terms.  A sphere leaf
// with RtLeaf::share_prev (the previous leaf of its object is a sphere with a bit-identical
// inverse transform and centre, and is evaluated by every lane that evaluates this one, see
// rt_blob.h) has the same object-space ray, hence the same 1/|d|, v.dn and v.v: only r^2 differs,
// so it reuses them and skips the transform, the length, the division and two dot products.
struct SphereShare { double il, vd, vv; };

template <bool POS = false>
__device__ __forceinline__ int leaf_candidates(cptr<RtLeaf> L, V3 ro, V3 rd, bool fin, double* t0, double* t1,
                                               SphereShare* sh = nullptr) {
#if RT_SPHERE_SHARE
  if (sh && L->share_prev) {                                               // math_shapes.rs:42-62
    const double sum = sh->vd * sh->vd - (sh->vv - L->r2);
    if (sum < 0.0) return 0;
    const double sq = sqrt_rt(sum);
    *t0 = (-sh->vd + sq) * sh->il;
    *t1 = (-sh->vd - sq) * sh->il;
    return 2;
  }
#endif
  V3 o, d;
  if (L->xdiag == RT_XF_IDENTITY && fin) {
    o = ro;
    d = rd;
  } else if (L->xdiag && fin) {                                            // transformation.rs:88-93
    o = xf_diag(L->inv, ro);
    d = sub(xf_diag(L->inv, rd), ld3(L->inv_o));
  } else {
    o = xf(L->inv, ro);
    d = sub(xf(L->inv, rd), ld3(L->inv_o));
  }
  int k = L->kind;
  if (k == RT_N_SPHERE) {                                                  // math_shapes.rs:42-62
    V3 v = sub(o, ld3(L->c));
    double l, il;
    len_inv(d, &l, &il);                                                   // il = 1.0 / len(d)
    V3 dn = scale(d, il);
    double vd = dot(v, dn);
    const double vv = dot(v, v);
    if (sh) *sh = {il, vd, vv};
    double sum = vd * vd - (vv - L->r2);
    if (sum < 0.0) return 0;
    double sq = sqrt_rt(sum);
    *t0 = (-vd + sq) * il;
    *t1 = (-vd - sq) * il;
    return 2;
  }
  if (k == RT_N_PLANE) {                                                   // :168-180
    V3 pn = ld3(L->pnorm);
    double v_d, num;
#if RT_PLANE_AXIS
    const int ax = L->plane_axis;
    if (POS && fin && ax >= 0) {               // axis-aligned normal: one product (rt_blob.h)
      if (ax == 0) { v_d = pn.x * d.x; num = pn.x * o.x; }
      else if (ax == 1) { v_d = pn.y * d.y; num = pn.y * o.y; }
      else { v_d = pn.z * d.z; num = pn.z * o.z; }
    } else
#endif
    {
      v_d = dot(pn, d);
      num = dot(pn, o);
    }
    if (v_d != 0.0) {
      num = num + L->pl[0][3];
      // t = -num * (1/v_d) is > 0 only if num and v_d have opposite signs (rounding keeps signs;
      // 1/v_d may overflow to +-inf, never to 0).  Otherwise t is <= 0, -0 or NaN: never > EPS.
      if (POS && !((num > 0.0 && v_d < 0.0) || (num < 0.0 && v_d > 0.0))) return 0;
      double t = -num * (1.0 / v_d);
      if (t >= 0.0) { *t0 = t; return 1; }
    }
    return 0;
  }
  double tn = -INFINITY, tf = INFINITY;                                    // :248-290
#define RT_SLAB(P, D, I)                                                    \
  if (D == 0.0) {                                                           \
    if (P < L->lo[I] || P > L->hi[I]) return 0;                             \
  } else {                                                                  \
    double a = (L->lo[I] - P) / D, b = (L->hi[I] - P) / D;                  \
    if (a > b) { double tmp = a; a = b; b = tmp; }                          \
    if (a > tn) tn = a;                                                     \
    if (b < tf) tf = b;                                                     \
    if (tn > tf || tf < 0.0) return 0;                                      \
  }
  RT_SLAB(o.x, d.x, 0)
  RT_SLAB(o.y, d.y, 1)
  RT_SLAB(o.z, d.z, 2)
#undef RT_SLAB
  *t0 = tn;
  *t1 = tf;
  return 2;
}

// Conjunction of every CSG ancestor's sibling test for a hit of leaf L at world point p
// (csg.rs:43-95), as a postfix program over a bit stack.
__device__ bool leaf_filter(const DS& S, cptr<RtLeaf> L, V3 p) {
  const bool fin = wave_finite(p);
  const int nl = L->n_lit;
  if (nl >= 0) {                                   // conjunction of literals (rt_blob.h)
    for (int k = 0; k < nl; ++k) {
      const int v = L->lit[k];
      if (leaf_inside(&S.leaves[v >> 1], p, fin) != (bool)(v & 1)) return false;
    }
    return true;
  }
  uint32_t st = 0;
  const int e = L->prog_end;
  for (int k = L->prog_begin; k < e; ++k) {
    const int op = S.prog[k].op, arg = S.prog[k].arg;
    if (op == RT_OP_INSIDE) {
      st = (st << 1) | (leaf_inside(&S.leaves[arg], p, fin) ? 1u : 0u);
    } else if (op == RT_OP_REQUIRE) {
      uint32_t v = st & 1u;
      st >>= 1;
      if (v != (uint32_t)arg) return false;
    } else {
      uint32_t b = st & 1u;
      st >>= 1;
      uint32_t a = st & 1u, r;
      if (op == RT_OP_AND) r = a & b;
      else if (op == RT_OP_OR) r = a | b;
      else r = a & (b ^ 1u);
      st = (st & ~1u) | r;
    }
  }
  return true;
}

// ------------------------------------------------------------------ conservative culling
// Does the ray segment t in [0, tmax] come near the box?  Only ever answers "no" when no point
// where an accepted hit could lie is on the segment.  Per axis the slab times are
// (bound - o) * inv with inv ~ 1/d to ~1e-15: for |origin|, |bounds| <= 1e6 the error in
// space is < 1e-9, far inside the 1e-6 inflation of every box (scene.cpp leaf_box), so each
// axis interval computed still contains the parameter of any point of the un-inflated region;
// tmax carries a 1e-7 relative margin on top.  min/max are IEEE minNum/maxNum: a NaN slab time
// narrows nothing, and a ray outside the proven range (cull_ray) gets NaN inv -> never culled.
struct CullRay { V3 inv, o; };

// Reciprocal for the culling slabs only (never for a value the reference computes): hardware
// rcp + one Newton step.  d == 0 (or |d| < 1e-200) -> +-1e200, which makes the slab test the
// "origin inside the slab" check while every product stays finite.
__device__ __forceinline__ double cull_rcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  const double n = fma(r, fma(-x, r, 1.0), r);
  return fabs(x) < 1e-200 ? copysign(1e200, x) : n;
}
__device__ __forceinline__ CullRay cull_ray(V3 o, V3 d) {
  const double ad = fmax(fmax(fabs(d.x), fabs(d.y)), fabs(d.z));
  const bool ok = fabs(o.x) <= RT_CULL_COORD_MAX && fabs(o.y) <= RT_CULL_COORD_MAX && fabs(o.z) <= RT_CULL_COORD_MAX &&
                  ad >= 1e-100 && ad <= 1e100;
  const double nan = __builtin_nan("");
  const V3 inv = ok ? V3{cull_rcp(d.x), cull_rcp(d.y), cull_rcp(d.z)} : V3{nan, nan, nan};
  return {inv, o};
}
// (bound - o) * inv per slab: measured faster than fma(bound, inv, -o*inv), which keeps three
// more doubles live across the traversal (profiles/r01n_variant_timing.txt).
template <class P> __device__ __forceinline__ bool box_may_hit(P lo, P hi, const CullRay& r, double tmax) {
  const double ax = (lo[0] - r.o.x) * r.inv.x, bx = (hi[0] - r.o.x) * r.inv.x;
  const double ay = (lo[1] - r.o.y) * r.inv.y, by = (hi[1] - r.o.y) * r.inv.y;
  const double az = (lo[2] - r.o.z) * r.inv.z, bz = (hi[2] - r.o.z) * r.inv.z;
  const double tn = fmax(fmax(fmin(ax, bx), fmin(ay, by)), fmax(fmin(az, bz), 0.0));
  const double tf = fmin(fmin(fmax(ax, bx), fmax(ay, by)), fmin(fmax(az, bz), tmax));
  return !(tn > tf);
}
__device__ __forceinline__ double cull_tmax(double t) { return t * (1.0 + 1e-7) + 1e-7; }

// The object's oriented box (RtObject::obb_leaf, scene.cpp obb): may the segment t in [0, tmax]
// meet the leaf-frame box olo/ohi?  The ray is taken to the leaf's frame with the leaves' own
// arithmetic; outside the range the host's margins are proven for (|o| <= 1e6, unit-length
// directions) the answer is yes.  The refraction kernels (SHARE: 4 waves/SIMD at 115-119 VGPRs)
// do not take it: the test's code alone made spinning_globes (no oriented box) 2.7 % slower
// (profiles/r02cg_obb_ab.txt).
#ifndef RT_OBB
#define RT_OBB 1
#endif
__device__ __forceinline__ bool obb_may_hit(const DS& S, cptr<RtObject> O, V3 ro, V3 rd, double tmax) {
  cptr<RtLeaf> R = &S.leaves[O->obb_leaf];
  const double ad = fmax(fmax(fabs(rd.x), fabs(rd.y)), fabs(rd.z));
  if (!(ad >= 0.25 && ad <= 4.0 && fabs(ro.x) <= 1e6 && fabs(ro.y) <= 1e6 && fabs(ro.z) <= 1e6)) return true;
  const V3 o = xf(R->inv, ro);
  const V3 d = sub(xf(R->inv, rd), ld3(R->inv_o));
  return box_may_hit(O->olo, O->ohi, cull_ray(o, d), tmax);
}

// ------------------------------------------------------------------ traversal (raytracer.rs)
// Both traversals walk the object hierarchy (RtTrav, pre-order over contiguous draw-order runs)
// wave-coherently: `i` is uniform, a lane that misses a group resumes at its skip index, and the
// wave jumps over a group no lane entered.  Objects are visited in draw order either way.

// Nearest hit over all objects in draw order: accept d if d > EPS && d < nearest
// (raytracer.rs:141-150).  The acceptance test is pure, so it runs BEFORE the (pure) CSG
// filter: candidates that cannot win never pay for the sibling is_inside tests.
// SHARE: concentric sphere leaves reuse their ray terms (SphereShare); it keeps three doubles live
// across the leaf loop, so only kernels with register headroom take it (see trace()).
template <bool SHARE = false, bool OBB = !SHARE>
__device__ int nearest_hit(const DS& S, V3 ro, V3 rd, double* dist, int cat = 0) {
  [[maybe_unused]] const int cb = cat * 9;
  CNT(cb + 0);
  CNTW(32 + cat);
  double best = INFINITY;
  int bobj = -1;
  SphereShare shr = {0.0, 0.0, 0.0};
  const CullRay cr = cull_ray(ro, rd);
  const bool fin = wave_finite(ro, rd);
  int resume = 0;
  // NORDER (reflection-only kernels): the objects in S.strav's order, largest regions first, so an
  // early hit on a big object culls what lies behind it.  Exact: a candidate equal to the best
  // distance so far wins when its object comes earlier in DRAW order (o < bobj), which is the
  // reference's first-visited-wins rule (raytracer.rs:141-150) for any visiting order.
  constexpr bool NORDER = RT_NEAREST_ORDER && OBB;
  const cptr<RtTrav> TR = NORDER ? S.strav : S.trav;
  const int n_tr = NORDER ? S.n_strav : S.n_trav;
  for (int i = 0; i < n_tr;) {
    cptr<RtTrav> T = &TR[i];
    const bool act = i >= resume;
    if (T->obj < 0) {                                    // group node
      CNT(28 + cat);
      const bool in = act && box_may_hit(T->blo, T->bhi, cr, cull_tmax(best));
      if (act && !in) resume = T->skip;
      i = __ballot(in) ? i + 1 : T->skip;
      continue;
    }
    ++i;
    if (!act) continue;
    // the object's cull kind and box come from the node's copy (RtTrav): one scalar load for the
    // node decides the common case; the object's own record is read only once its box passes
    if (T->cull == RT_CULL_ALWAYS) continue;
    if (T->cull == RT_CULL_BOX) CNT(cb + 1);
    if (T->cull == RT_CULL_BOX && !box_may_hit(T->blo, T->bhi, cr, cull_tmax(best))) continue;
    const int o = T->obj;
    cptr<RtObject> O = &S.objects[o];
    if (RT_OBB && OBB && O->obb_leaf >= 0 && !obb_may_hit(S, O, ro, rd, cull_tmax(best))) continue;
    CNT(cb + 2);
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    for (int l = lb; l < le; ++l) {
      cptr<RtLeaf> L = &S.leaves[l];
      if (O->leaf_cull) {
        if (L->cull == RT_CULL_ALWAYS) continue;
        if (L->cull == RT_CULL_BOX) CNT(cb + 3);
        if (L->cull == RT_CULL_BOX && !box_may_hit(L->blo, L->bhi, cr, cull_tmax(best))) continue;
      }
      CNT(cb + 4);
      CNT(40 + cat * 8 + (o & 7));                      // per-object leaf evaluations (diagnostic)
      CNTW(35 + cat);
      CNT(cb + 5 + (L->kind == RT_N_SPHERE ? 0 : L->kind == RT_N_PLANE ? 1 : 2));
      double t0 = 0.0, t1 = 0.0;
      int n = leaf_candidates<true>(L, ro, rd, fin, &t0, &t1, SHARE ? &shr : nullptr);
      const bool filtered = L->prog_end != L->prog_begin && !(RT_CONST_FILTER && SHARE && L->filter_const && !isnan(cr.inv.x));
      if (filtered && ((n >= 1 && t0 > EPS && t0 < best) || (n >= 2 && t1 > EPS))) CNT(cb + 8);
      if (n >= 1 && t0 > EPS && (t0 < best || (NORDER && t0 == best && o < bobj)) &&
          (!filtered || leaf_filter(S, L, add(ro, scale(rd, t0))))) {
        best = t0; bobj = o;
      }
      if (n >= 2 && t1 > EPS && (t1 < best || (NORDER && t1 == best && o < bobj)) &&
          (!filtered || leaf_filter(S, L, add(ro, scale(rd, t1))))) {
        best = t1; bobj = o;
      }
    }
  }
  *dist = best;
  return bobj;
}

// Product of the transparencies of every filtered hit with EPS < d < dist (raytracer.rs:181-197).
// Early-out once the product is exactly 0 (it stays 0: every factor is finite, checked on the
// host), objects of transparency exactly 1.0 are skipped (x * 1.0 == x).
// SORDER (reflection-only kernels): walk S.strav, the likeliest occluders first (scene.cpp
// shadow_order) -- every transparency is +-0 there, so the first filtered hit decides and the
// order is free.
template <bool SHARE = false, bool OBB = !SHARE, bool SORDER = OBB>
__device__ double shadow_transparency(const DS& S, V3 p, V3 dir, double dist) {
  [[maybe_unused]] constexpr int cb = 18;
  CNT(cb + 0);
  CNTW(34);
  double tr = 1.0;
  SphereShare shr = {0.0, 0.0, 0.0};
  const CullRay cr = cull_ray(p, dir);
  const bool fin = wave_finite(p, dir);
  const double tmax = cull_tmax(dist);
  int resume = 0;
  const cptr<RtTrav> TR = (RT_SHADOW_ORDER && SORDER) ? S.strav : S.trav;
  const int n_tr = (RT_SHADOW_ORDER && SORDER) ? S.n_strav : S.n_trav;
  for (int i = 0; i < n_tr;) {
    cptr<RtTrav> T = &TR[i];
    const bool act = i >= resume;
    if (T->obj < 0) {                                    // group node
      CNT(30);
      const bool in = act && box_may_hit(T->blo, T->bhi, cr, tmax);
      if (act && !in) resume = T->skip;
      i = __ballot(in) ? i + 1 : T->skip;
      continue;
    }
    ++i;
    if (!act) continue;
    if (T->shadow_skip || T->cull == RT_CULL_ALWAYS) continue;     // the node's copies (see nearest_hit)
    if (T->cull == RT_CULL_BOX) CNT(cb + 1);
    if (T->cull == RT_CULL_BOX && !box_may_hit(T->blo, T->bhi, cr, tmax)) continue;
    cptr<RtObject> O = &S.objects[T->obj];
    if (RT_OBB && OBB && O->obb_leaf >= 0 && !obb_may_hit(S, O, p, dir, tmax)) continue;
    CNT(cb + 2);
    const double tobj = O->transparency;
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    for (int l = lb; l < le; ++l) {
      cptr<RtLeaf> L = &S.leaves[l];
      if (O->leaf_cull) {
        if (L->cull == RT_CULL_ALWAYS) continue;
        if (L->cull == RT_CULL_BOX) CNT(cb + 3);
        if (L->cull == RT_CULL_BOX && !box_may_hit(L->blo, L->bhi, cr, tmax)) continue;
      }
      CNT(cb + 4);
      CNT(56 + (T->obj & 7));
      CNTW(37);
      CNT(cb + 5 + (L->kind == RT_N_SPHERE ? 0 : L->kind == RT_N_PLANE ? 1 : 2));
      double t0 = 0.0, t1 = 0.0;
      int n = leaf_candidates<true>(L, p, dir, fin, &t0, &t1, SHARE ? &shr : nullptr);
      const bool filtered = L->prog_end != L->prog_begin && !(RT_CONST_FILTER && SHARE && L->filter_const && !isnan(cr.inv.x));
      if (filtered && ((n >= 1 && t0 > EPS && t0 < dist) || (n >= 2 && t1 > EPS && t1 < dist))) CNT(cb + 8);
      if (n >= 1 && t0 > EPS && t0 < dist && (!filtered || leaf_filter(S, L, add(p, scale(dir, t0))))) {
        tr *= tobj;
        if (tr == 0.0 && S.shadow_early_out) return 0.0;
      }
      if (n >= 2 && t1 > EPS && t1 < dist && (!filtered || leaf_filter(S, L, add(p, scale(dir, t1))))) {
        tr *= tobj;
        if (tr == 0.0 && S.shadow_early_out) return 0.0;
      }
    }
  }
  return tr;
}

// Normal and UV of top-level object O at point p: RTObject shape get_normal / get_uv_coordinates,
// with CSG's is_on_surface / is_inside evaluated bottom-up over the post-order node list
// (csg.rs:98-168) and the descent a-then-b of csg.rs:104-121 / :161-167.
__device__ void object_normal_uv(const DS& S, cptr<RtObject> O, V3 p, bool want_uv, V3* n,
                                 double* u, double* v) {
  cptr<RtNode> N = S.nodes + O->node_begin;
  const int cnt = O->node_count;
  const bool fin = wave_finite(p);
  *u = 0.0;
  *v = 0.0;
  if (cnt == 1) {
    cptr<RtLeaf> L = &S.leaves[N[0].leaf];
    *n = leaf_normal(L, p, fin);
    if (want_uv && L->kind == RT_N_SPHERE) sphere_uv(L, p, u, v);
    return;
  }
  uint32_t in = 0, on = 0;
  for (int i = 0; i < cnt; ++i) {
    const int nk = N[i].kind, na = N[i].a, nb = N[i].b, nl = N[i].leaf;
    bool bi, bo;
    if (nk < RT_N_UNION) {
      cptr<RtLeaf> L = &S.leaves[nl];
      bi = leaf_inside(L, p, fin);
      bo = leaf_on_surface(L, p, fin);
    } else {
      bool ia = (in >> na) & 1u, ib = (in >> nb) & 1u, oa = (on >> na) & 1u, ob = (on >> nb) & 1u;
      if (nk == RT_N_UNION) { bi = ia || ib; bo = (oa && !ib) || (ob && !ia); }
      else if (nk == RT_N_INTERSECTION) { bi = ia && ib; bo = (oa && ib) || (ob && ia); }
      else { bi = ia && !ib; bo = (oa && !ib) || (ob && ia); }
    }
    in |= (uint32_t)bi << i;
    on |= (uint32_t)bo << i;
  }
  // Descent a-then-b (csg.rs:104-121, :161-167).  Children precede parents in post-order, so one
  // downward pass over the node indices visits every lane's path in order; node reads stay
  // wave-uniform (scalar).  Membership tests go through ballot masks (see trace()).
  const int lane = __lane_id();
  int cur = cnt - 1, sel = -1;
  bool neg = false;
  for (int i = cnt - 1; i >= 0; --i) {
    const int nk = N[i].kind, na = N[i].a, nb = N[i].b, nl = N[i].leaf;
    if (!((__ballot(cur == i) >> lane) & 1)) continue;
    if (nk < RT_N_UNION) { sel = nl; cur = -1; }
    else if ((on >> na) & 1u) cur = na;
    else if ((on >> nb) & 1u) { if (nk == RT_N_DIFFERENCE) neg = !neg; cur = nb; }   // b.get_normal(p) * -1.0
    else cur = -1;                                          // fallback (1,0,0); UV is Err -> (0,0)
  }
  *n = {1.0, 0.0, 0.0};
  const int lb = O->leaf_begin, le = lb + O->leaf_count;
  for (int l = lb; l < le; ++l) {
    if (!((__ballot(sel == l) >> lane) & 1)) continue;
    cptr<RtLeaf> L = &S.leaves[l];
    *n = leaf_normal(L, p, fin);
    if (want_uv && L->kind == RT_N_SPHERE) sphere_uv(L, p, u, v);
  }
  if (neg) *n = scale(*n, -1.0);
}

// PixmapTexture::get_color_at (texture.rs:27-34) on RGBA8 texels, /255.0 (sceneparser/texture.rs:29-33)
__device__ Col texture_color(const DS& S, int tex, double u, double v) {
  const int tw = S.textures[tex].w, th = S.textures[tex].h;
  const int64_t toff = S.textures[tex].offset;
  double x = u * (double)(tw - 1);
  double y = (double)th - (v * (double)(th - 1)) - 1.0;
  // `as usize` saturates (NaN/negative -> 0); the reference would panic past the edge: clamp.
  int xi = x > 0.0 ? (x < (double)(tw - 1) ? (int)x : tw - 1) : 0;
  int yi = y > 0.0 ? (y < (double)(th - 1) ? (int)y : th - 1) : 0;
  const uint32_t px = *(const uint32_t*)(S.texels + toff + ((size_t)yi * tw + xi) * 4);
  return {(double)(px & 0xffu) / 255.0, (double)((px >> 8) & 0xffu) / 255.0, (double)((px >> 16) & 0xffu) / 255.0};
}

// angle(-dir, n) >= PI/2 (raytracer.rs:230-231) from the cosine `cin` the angle's acos would take
// (vector.rs:57-59).  acos is monotone and rt_acos is within 1 ulp, so for |cin| > 1e-15 (>= 4 ulp
// of PI/2 away from the threshold) the sign decides exactly -- except past -1: a cosine that
// rounds below -1 (a ray through a sphere's centre meets the normal head-on) makes acos NaN and
// the comparison false, so such a hit is NOT inside.  Near-grazing cosines (and NaN) evaluate
// the acos itself.
__device__ __forceinline__ bool inside_test(double cin) {
  return cin < -1e-15 ? cin >= -1.0 : (cin > 1e-15 ? false : rt_acos(cin) >= PI_D / 2.0);
}

__device__ __forceinline__ V3 reflect_dir(V3 i, V3 n) {                    // raytracer.rs:332-334
  return sub(i, scale(scale(n, 2.0), dot(n, i)));
}
__device__ __forceinline__ V3 refract_dir(V3 i, V3 n, double r, bool* tir) {   // raytracer.rs:336-353
  double cos_1 = dot(scale(i, -1.0), n);
  double v = 1.0 - r * r * (1.0 - cos_1 * cos_1);
  *tir = v < 0.0;
  if (*tir) return {0.0, 0.0, 0.0};
  double cos_2 = sqrt_rt(v);
  return normalized(add(scale(i, r), scale(n, r * cos_1 - cos_2)));
}

// Normal (normalised, :163), material colour at the UV (:165-170), transparency, reflectivity of
// each lane's hit object -- SCALARISED over the distinct objects hit in this wave (readlane of the
// first remaining lane), so every object / node / leaf read is wave-uniform (SMEM, no VGPRs).
__device__ __forceinline__ void shade_inputs(const DS& S, int oi, V3 p, V3* nrm, Col* c, double* transp,
                                             double* refl) {
  uint64_t todo = __ballot(oi >= 0);
  while (todo) {
    CNTW(27);
    const int o = __builtin_amdgcn_readlane(oi, (int)__builtin_ctzll(todo));
    const uint64_t mine = __ballot(oi == o);
    todo &= ~mine;
    // test membership through the ballot mask, not `oi == o`: an equality lets the optimiser
    // substitute the per-lane oi for the uniform o and the loads below turn into VMEM again.
    if ((mine >> __lane_id()) & 1) {
      cptr<RtObject> O = &S.objects[o];
      double u, v;
      object_normal_uv(S, O, p, O->textured != 0, nrm, &u, &v);
      *c = O->textured ? texture_color(S, O->tex, u, v) : Col{O->color[0], O->color[1], O->color[2]};
      *transp = O->transparency;
      *refl = O->reflectivity;
    }
  }
  *nrm = normalized(*nrm);
}

using RtRayRecord = rt_ray_record;

// Ray-debugger recording (raytracer.rs:17-19, :155-157, :282-284; ray_debugger.rs:92-137).
// NoRec compiles to nothing in the render kernels; RtRayRecord slots are written in ray START
// order and `order` lists them in the reference's callback order (a ray reports after its
// children: post-order).
struct NoRec {
  __device__ __forceinline__ int begin(int, int, V3, V3, double, int, V3) { return 0; }
  __device__ __forceinline__ void finish(int, Col) {}
};
struct BufRec {
  RtRayRecord* rec;
  int* order;
  int cap, n_begun, n_done;
  const DS* S;
  __device__ int begin(int depth, int type, V3 ro, V3 rd, double t, int oi, V3 p) {
    const int i = n_begun++;
    if (i >= cap) return -1;
    RtRayRecord& r = rec[i];
    r.depth = depth; r.ray_type = type; r.object = oi; r.intersected = t != INFINITY;
    r.point[0] = ro.x; r.point[1] = ro.y; r.point[2] = ro.z;
    r.direction[0] = rd.x; r.direction[1] = rd.y; r.direction[2] = rd.z;
    r.distance = t;
    const V3 ip = add(ro, scale(rd, r.intersected ? t : 1000.0));          // ray_debugger.rs:107-111
    r.intersection[0] = ip.x; r.intersection[1] = ip.y; r.intersection[2] = ip.z;
    r.has_normal = oi >= 0;
    V3 n = {0.0, 0.0, 0.0};
    if (oi >= 0) {                                                         // shape.get_normal (:113-119)
      double u, v;
      object_normal_uv(*S, &S->objects[oi], ip, false, &n, &u, &v);
    }
    r.normal[0] = n.x; r.normal[1] = n.y; r.normal[2] = n.z;
    return i;
  }
  __device__ void finish(int i, Col c) {
    if (i < 0) return;
    rec[i].color[0] = c.r; rec[i].color[1] = c.g; rec[i].color[2] = c.b; rec[i].color[3] = 1.0;
    if (n_done < cap) order[n_done] = i;
    ++n_done;
  }
};

// Frame-stack slots in LDS.  The first KL frames of every lane's stack (A.r, A.g, A.b, w) live in
// LDS laid out [frame][component][lane], so each access is one conflict-free ds_*_b64; deeper
// frames (chains longer than KL, rare) use the private array, i.e. scratch.  KL = 2: 4 KB per
// one-wave workgroup, 80 of the 160 KB at 5 waves/SIMD.  With the megakernel at 5 waves/SIMD
// (below) the stack was the last large source of scratch traffic: KL = 2 cuts the 4K globes
// launch's HBM traffic from 0.245 to 0.105 GB (writes 0.21 -> 0.082 GB, 2.5x the 33 MB frame) at
// equal time (+0.4 %, noise; KL = 4: 0.089 GB but 5 % slower), profiles/r02t_*.  (At 7 waves/SIMD,
// round 1, KL = 4 measured 0.2-0.8 % slower than the scratch stack, profiles/r01r_lds_stack_ab.txt.)
#define LDS_AS __attribute__((address_space(3)))
typedef LDS_AS double lds_f64;
#ifndef RT_LDS_FRAMES
#define RT_LDS_FRAMES 2
#endif
// Refraction-chain kernels (RT_MODE_CHAIN): frames of the chain stack kept in LDS.  At 4 waves/SIMD
// (below) 5 frames fill the 160 KB of a CU (10 KB per one-wave workgroup).
#ifndef RT_LDS_FRAMES_CHAIN
#define RT_LDS_FRAMES_CHAIN 5
#endif
// Refraction frames also carry the pending reflection ray (P, D, rp: 7 doubles); the first
// KLR of them go to LDS after the KL colour frames, [frame][component][lane] likewise.
#ifndef RT_LDS_RFRAMES
#define RT_LDS_RFRAMES 1
#endif

// get_ray_color (raytracer.rs:132-287) for one primary ray, recursion unrolled onto a per-lane
// frame stack.  REFR = the scene has a transparent object (refraction frames need more state).
// KL > 0: frames 0..KL-1 of the stack are in LDS at lf[(f * 4 + c) * 64] (lf = this lane's slot);
// KLR > 0 (REFR): the pending-reflection state of frames 0..KLR-1 at lf[(KL * 4 + f * 7 + c) * 64].
// CHAIN (REFR scenes with RtDevScene::ray_chains): every hit spawns at most one ray, so a refraction
// frame never carries a pending reflection: frames are (A, w) as in the reflection-only kernels.
template <bool REFR, class Rec = NoRec, int KL = 0, bool FC = false, int KLR = 0, bool CHAIN = false>
__device__ Col trace(const DS& S, V3 ro, V3 rd, int max_depth, Rec* rec = nullptr, lds_f64* lf = nullptr) {
  double fA[RT_MAX_DEPTH_CAP][3];     // parent colour already intensified by (1 - w)
  double fW[RT_MAX_DEPTH_CAP];        // child weight w (transparency or reflectivity)
  auto put_frame = [&](int f, Col A, double w) {
    if (KL > 0 && f < KL) {
      lf[(f * 4 + 0) * 64] = A.r; lf[(f * 4 + 1) * 64] = A.g; lf[(f * 4 + 2) * 64] = A.b; lf[(f * 4 + 3) * 64] = w;
    } else {
      fA[f][0] = A.r; fA[f][1] = A.g; fA[f][2] = A.b; fW[f] = w;
    }
  };
  auto get_frame = [&](int f, Col* A, double* w) {
    if (KL > 0 && f < KL) {
      *A = {lf[(f * 4 + 0) * 64], lf[(f * 4 + 1) * 64], lf[(f * 4 + 2) * 64]}; *w = lf[(f * 4 + 3) * 64];
    } else {
      *A = {fA[f][0], fA[f][1], fA[f][2]}; *w = fW[f];
    }
  };
  constexpr bool TREE = REFR && !CHAIN;       // a hit may spawn two rays: pending reflections
  double fP[TREE ? RT_MAX_DEPTH_CAP : 1][3], fD[TREE ? RT_MAX_DEPTH_CAP : 1][3];
  double fRP[TREE ? RT_MAX_DEPTH_CAP : 1];
  uint32_t pend = 0;                  // bit f: frame f's reflection ray is still to be traced
  static_assert(RT_MAX_DEPTH_CAP <= 32, "pending-reflection bit mask");
  auto put_rframe = [&](int f, V3 P, V3 D, double rp) {
    if (KLR > 0 && f < KLR) {
      lds_f64* q = lf + (KL * 4 + f * 7) * 64;
      q[0] = P.x; q[64] = P.y; q[128] = P.z; q[192] = D.x; q[256] = D.y; q[320] = D.z; q[384] = rp;
    } else {
      fP[f][0] = P.x; fP[f][1] = P.y; fP[f][2] = P.z; fD[f][0] = D.x; fD[f][1] = D.y; fD[f][2] = D.z; fRP[f] = rp;
    }
  };
  auto get_rframe = [&](int f, V3* P, V3* D, double* rp) {
    if (KLR > 0 && f < KLR) {
      const lds_f64* q = lf + (KL * 4 + f * 7) * 64;
      *P = {q[0], q[64], q[128]}; *D = {q[192], q[256], q[320]}; *rp = q[384];
    } else {
      *P = {fP[f][0], fP[f][1], fP[f][2]}; *D = {fD[f][0], fD[f][1], fD[f][2]}; *rp = fRP[f];
    }
  };
  constexpr bool RECORD = !std::is_same<Rec, NoRec>::value;
  // Shared sphere terms (SphereShare) in the refraction kernels only: at 4 waves/SIMD they have
  // the registers (104 -> 116 VGPRs, no spill; spinning_globes 1080p 4.8 % faster), while the
  // reflection-only megakernel at 5 waves spills 14 more VGPRs and runs 6 % slower on 4K globes
  // (profiles/r02am_ab.txt).
  constexpr bool SHARE = REFR && RT_SPHERE_SHARE && (!CHAIN || RT_SPHERE_SHARE_CHAIN);
  constexpr bool OBB = !REFR;                          // oriented object boxes: reflection-only kernels
  int fSlot[RECORD ? RT_MAX_DEPTH_CAP : 1];
  [[maybe_unused]] int ray_type = 0, slot = 0;                  // RayType::NormalRay
  int sp = 0, depth = 0;
  Col C = {0.0, 0.0, 0.0};
  [[maybe_unused]] int trip = 0;
  for (;;) {
    bool descend = false;
    double t_hit;
    PROF_T0(p0);
    const int oi = nearest_hit<SHARE, OBB>(S, ro, rd, &t_hit, trip == 0 ? 0 : 1);
    PROF_ADD(trip == 0 ? 0 : 1, p0);
    ++trip;
    PROF_T0(p1);
#ifdef RT_ABLATE_TRAVERSAL_ONLY          // diagnostic builds only (tools/ablation): cost split
    return Col{t_hit * 1e-3, (double)oi, 0.0};
#endif
    const V3 p = add(ro, scale(rd, t_hit));                               // :162
    if constexpr (RECORD) slot = rec->begin(depth, ray_type, ro, rd, t_hit, oi, p);
    V3 nrm = {0.0, 0.0, 0.0};
    Col c = {0.0, 0.0, 0.0}, L = {0.0, 0.0, 0.0};
    double transp = 0.0, refl = 0.0;
    if (oi >= 0) {
      // Evaluation order is free (every step is a pure function of the hit), so the shadow
      // rays of a group of lights are traced FIRST, while only the hit point is live, and the
      // normal / UV / material and the per-light Lambert terms are formed afterwards: far fewer
      // registers live across the traversals.  Light accumulation order is unchanged.
      bool have_shading = false;
      // One light at a time: the unit vector towards the light is the shadow ray's direction
      // (:176-178) AND the Lambert term's `sdir` (:203-205), the same operations on the same
      // operands, so it is formed once and kept for the Lambert term.
#pragma unroll 1
      for (int k = 0; k < S.n_lights; ++k) {
        cptr<RtLight> lt = &S.lights[k];
        const V3 lv = sub(ld3(lt->p), p);
        double ll, ill;
        len_inv(lv, &ll, &ill);
        const V3 sdir = scale(lv, ill);                                    // normalized(lv)
#ifdef RT_ABLATE_NO_SHADOWS
        const double t = lv.x > 1e300 ? 0.5 : 1.0;
#else
        PROF_T0(p2);
        const double t = shadow_transparency<SHARE, OBB>(S, p, sdir, ll);       // :176-197
        PROF_ADD(2, p2);
#endif
        if (!have_shading) {
          PROF_T0(p3);
          shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);
          PROF_ADD(3, p3);
          L = cmul<FC>(c, in_range<FC>(0.6, 0.6, 0.6));                      // ambient (:172)
          have_shading = true;
        }
        if (t == 0.0) continue;                                            // :199-227
        double ang = rt_acos(dot(sdir, nrm) / (len(sdir) * len(nrm)));
        if (ang >= PI_D / 2.0) ang = PI_D - ang;
        const double inten = (ang < (PI_D / 2.0) && ang >= 0.0) ? 1.0 - (ang / (PI_D / 2.0)) : 0.0;
        const Col lc = intensify<FC>(intensify<FC>(Col{lt->col[0], lt->col[1], lt->col[2]}, inten), t);
        L = cadd<FC>(L, cmul<FC>(c, lc));
      }
      if (!have_shading) {
        shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);
        L = cmul<FC>(c, in_range<FC>(0.6, 0.6, 0.6));
      }
    }
    if (oi < 0) {
      C = {0.0, 0.0, 0.0};                                               // Color::BLACK (:152-160)
    } else {
      // The inside test (:230-235) only matters for a hit that spawns a ray: one with
      // depth < max_depth and a reflectivity or a transparency.  Other hits skip its division
      // and square roots (the values it would give are never read).
      bool inside = false;
      if (depth < max_depth && (refl != 0.0 || (REFR && transp != 0.0))) {
        const V3 nd = scale(rd, -1.0);
        inside = inside_test(dot(nd, nrm) / (len(nd) * len(nrm)));
      }
      const V3 n2 = inside ? scale(nrm, -1.0) : nrm;
      const double r1 = inside ? 1.45 : 1.0, r2 = inside ? 1.0 : 1.45;
      bool tir = false;
      V3 tdir = {0.0, 0.0, 0.0};
      const bool do_refr = REFR && depth < max_depth && transp != 0.0;   // :242
      if (do_refr) tdir = refract_dir(rd, n2, r1 / r2, &tir);
      const double rp = tir ? refl + (1.0 - refl) * transp : refl;       // :261-265
      const bool do_refl = depth < max_depth && rp != 0.0 && (!inside || tir);   // :267
      if (do_refr && !tir) {
        put_frame(sp, intensify<FC>(L, 1.0 - transp), transp);
        if constexpr (TREE) {
          pend = do_refl ? pend | (1u << sp) : pend & ~(1u << sp);
          if (do_refl) put_rframe(sp, p, reflect_dir(rd, n2), rp);
        }                                                                  // CHAIN: do_refl is false here
        if constexpr (RECORD) { fSlot[sp] = slot; ray_type = 2; }        // TransmissionRay
        ++sp;
        ro = p;
        rd = tdir;
        depth = sp;
        descend = true;
      } else if (do_refl) {
        put_frame(sp, intensify<FC>(L, 1.0 - rp), rp);
        if constexpr (TREE) pend &= ~(1u << sp);
        if constexpr (RECORD) { fSlot[sp] = slot; ray_type = 1; }        // ReflectionRay
        ++sp;
        rd = reflect_dir(rd, n2);
        ro = p;
        depth = sp;
        descend = true;
      } else {
        C = L;
      }
    }
    if constexpr (RECORD) { if (!descend) rec->finish(slot, C); }     // leaf ray (or miss) reports now
    PROF_ADD(4, p1);
    if (descend) continue;
    while (sp > 0) {                                                      // post-order combine
      const int f = sp - 1;
      Col fa;
      double fw;
      get_frame(f, &fa, &fw);
      const Col comb = cadd<FC>(fa, intensify<FC>(C, fw));
      if constexpr (TREE) {
        if ((pend >> f) & 1u) {                                           // refraction done -> reflection
          pend &= ~(1u << f);
          double frp;
          get_rframe(f, &ro, &rd, &frp);
          put_frame(f, intensify<FC>(comb, 1.0 - frp), frp);
          depth = sp;
          descend = true;
          if constexpr (RECORD) ray_type = 1;                              // ReflectionRay
          break;
        }
      }
      C = comb;
      if constexpr (RECORD) rec->finish(fSlot[f], C);                  // parent reports after its children
      --sp;
    }
    if (!descend) return C;
  }
}

// ---------------------------------------------------------------- deferred shadows (REFR=false)
// get_ray_color (raytracer.rs:132-287) for scenes without a transparent object, restructured so
// a pixel's critical path is its chain of nearest hits rather than nearest hits AND every shadow
// ray in series.  Without refraction every hit spawns at most one ray (the reflection), so a
// pixel's rays form a chain and the reference's recursion computes
//     C_h = L_h                                            (no reflection spawned)
//     C_h = in_range(in_range(L_h * (1 - w_h)) + in_range(C_{h+1} * w_h))      (:267-280)
// with L_h = the ambient + per-light Lambert terms of hit h (:172-228) and C = BLACK for a ray
// that misses (:152-160).  Every L_h is a pure function of hit h and its lights' shadow
// transparencies, so the three steps run as phases of one wave:
//   1. chain:   per lane, trace the nearest-hit chain; per hit record p, the normal, the material
//               colour and the reflection weight w in the lane's arrays (every hit but possibly
//               the last spawned a reflection);
//   2. shadows: every (hit, light) shadow ray of the WHOLE WAVE is dealt densely over its 64
//               lanes through an LDS window (one round = up to 64 hits; the hits' owners write
//               their points, any lane traces any (hit, light) pair, the owners read the
//               transparencies back and form L_h in light order, :199-227);
//   3. fold:    per lane, C from the last hit back to the first, the post-order combine.
// Same operations, same order per value: bit-identical to trace<false>.  A pixel whose chain is
// 11 bounces long now waits for 11 nearest-hit traversals plus a few dense shadow rounds, not
// 11 * (1 + lights) serial traversals; lanes whose chains ended early trace other lanes' shadow
// rays instead of idling.
#ifndef RT_SH_TRCAP
#define RT_SH_TRCAP 128             // shadow results per round: hits per round = min(64, TRCAP / lights)
#endif
#define RT_SPLIT_TILE_MASK 0xFFFFFu   // order entries: tile index in bits 0-19 (split tiles: see below)
#ifndef RT_SPLIT_MAX_LOG2
#define RT_SPLIT_MAX_LOG2 3           // a costly tile goes to at most 2^3 = 8 waves (part: bits 20-23)
#endif
static_assert(RT_SPLIT_MAX_LOG2 <= 4, "split part index has 4 bits");
struct ShadowWin {                  // LDS, one per wave: 2.5 KB
  double px[64], py[64], pz[64];
  double tr[RT_SH_TRCAP];
};

#ifdef RT_TILE_STATS                // diagnostic build only: per-tile phase times and chain lengths
#define RT_STATS_TILES (1 << 18)
__device__ uint32_t g_tile_stats[RT_STATS_TILES][4];
#endif

// REFR (scenes with RtDevScene::ray_chains and a transparent object): a hit spawns a refraction
// ray (weight transparency) or, on TIR or for a reflective object, a reflection ray (weight rp,
// raytracer.rs:261-265), never both, so the rays still form a chain and the same three phases
// apply; the decisions, directions and weights are trace<true, ..., CHAIN>'s, the traversals take
// the refraction kernels' template arguments (shared sphere terms, draw-order shadow walk: the
// transparency product's order is the reference's).
template <int HC, bool FC = false, bool REFR = false>
__device__ Col trace_deferred(const DS& S, V3 ro, V3 rd, int max_depth, bool valid, ShadowWin* win,
                              [[maybe_unused]] int stats_tile = -1) {
  constexpr bool SHARE = REFR && RT_SPHERE_SHARE, OBB = !REFR;
#ifdef RT_TILE_STATS
  const uint64_t ts0 = wall_clock64();
  int rounds = 0;
#endif
  double hP[HC][3], hN[HC][3], hC[HC][3], hW[HC];
  int nh = 0;
  bool last_spawned = false;          // the last hit spawned a reflection ray (that missed)
  // ---- phase 1: the nearest-hit chain
  if (valid) {
    for (int depth = 0;; ++depth) {
      double t_hit;
      const int oi = nearest_hit<SHARE, OBB>(S, ro, rd, &t_hit, depth == 0 ? 0 : 1);
      if (oi < 0) break;                                                   // BLACK (:152-160)
      const V3 p = add(ro, scale(rd, t_hit));                               // :162
      V3 nrm;
      Col c;
      double transp, refl;
      shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);                    // :163-170
      // inside test (:230-235), exactly as trace(): needed only if a ray may spawn
      bool inside = false;
      if (depth < max_depth && (refl != 0.0 || (REFR && transp != 0.0))) {
        const V3 nd = scale(rd, -1.0);
        inside = inside_test(dot(nd, nrm) / (len(nd) * len(nrm)));
      }
      const V3 n2 = inside ? scale(nrm, -1.0) : nrm;
      bool tir = false;
      V3 tdir = {0.0, 0.0, 0.0};
      const bool do_refr = REFR && depth < max_depth && transp != 0.0;     // :242
      const double r1 = inside ? 1.45 : 1.0, r2 = inside ? 1.0 : 1.45;
      if (do_refr) tdir = refract_dir(rd, n2, r1 / r2, &tir);
      const double rp = tir ? refl + (1.0 - refl) * transp : refl;         // :261-265
      const bool refracts = do_refr && !tir;
      const bool do_refl = !refracts && depth < max_depth && rp != 0.0 && (!inside || tir);   // :267
      hP[nh][0] = p.x; hP[nh][1] = p.y; hP[nh][2] = p.z;
      hN[nh][0] = nrm.x; hN[nh][1] = nrm.y; hN[nh][2] = nrm.z;
      hC[nh][0] = c.r; hC[nh][1] = c.g; hC[nh][2] = c.b;
      hW[nh] = refracts ? transp : rp;
      ++nh;
      last_spawned = refracts || do_refl;
      if (!last_spawned) break;
      rd = refracts ? tdir : reflect_dir(rd, n2);
      ro = p;
    }
  }
  // ---- phase 2: every shadow ray of the wave, dealt over all 64 lanes
  const int lane = __lane_id();
#ifdef RT_TILE_STATS
  const uint64_t ts1 = wall_clock64();
  int mx = nh, sm = nh;
  for (int d = 32; d >= 1; d >>= 1) { mx = max(mx, __shfl_xor(mx, d)); sm += __shfl_xor(sm, d); }
#endif
  const int nl = S.n_lights;
  const int hpr = nl > 0 ? (RT_SH_TRCAP / nl < 64 ? RT_SH_TRCAP / nl : 64) : 64;
  for (int next = 0;;) {
    const int pend = nh - next;
    int incl = pend;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const int total = __shfl(incl, 63);
    if (total == 0) break;                                                  // wave-uniform
    const int base = incl - pend;
    const int take = base >= hpr ? 0 : (pend < hpr - base ? pend : hpr - base);
    for (int i = 0; i < take; ++i) {
      win->px[base + i] = hP[next + i][0];
      win->py[base + i] = hP[next + i][1];
      win->pz[base + i] = hP[next + i][2];
    }
    const int n_pub = total < hpr ? total : hpr;
#ifdef RT_TILE_STATS
    ++rounds;
#endif
    __syncthreads();
    const int jobs = n_pub * nl;
    for (int j = lane; j < jobs; j += 64) {                                 // :176-197
      const int h = j % n_pub, k = j / n_pub;
      const V3 p = {win->px[h], win->py[h], win->pz[h]};
      const V3 lv = sub(ld3(S.lights[k].p), p);
      win->tr[j] = shadow_transparency<SHARE, OBB, OBB>(S, p, normalized(lv), len(lv));
    }
    __syncthreads();
    for (int i = 0; i < take; ++i) {                                        // L_h in light order
      const int hh = next + i;
      const V3 p = {hP[hh][0], hP[hh][1], hP[hh][2]};
      const V3 nrm = {hN[hh][0], hN[hh][1], hN[hh][2]};
      const Col c = {hC[hh][0], hC[hh][1], hC[hh][2]};
      Col L = cmul<FC>(c, in_range<FC>(0.6, 0.6, 0.6));                             // ambient (:172)
      for (int k = 0; k < nl; ++k) {                                        // :199-227
        const double tr = win->tr[k * n_pub + base + i];
        if (tr == 0.0) continue;
        cptr<RtLight> lt = &S.lights[k];
        const V3 sdir = normalized(sub(ld3(lt->p), p));
        double ang = rt_acos(dot(sdir, nrm) / (len(sdir) * len(nrm)));
        if (ang >= PI_D / 2.0) ang = PI_D - ang;
        const double inten = (ang < (PI_D / 2.0) && ang >= 0.0) ? 1.0 - (ang / (PI_D / 2.0)) : 0.0;
        const Col lc = intensify<FC>(intensify<FC>(Col{lt->col[0], lt->col[1], lt->col[2]}, inten), tr);
        L = cadd<FC>(L, cmul<FC>(c, lc));
      }
      hC[hh][0] = L.r; hC[hh][1] = L.g; hC[hh][2] = L.b;
    }
    next += take;
    __syncthreads();                                                        // the window is reused
  }
  // ---- phase 3: post-order combine, last hit first
#ifdef RT_TILE_STATS
  const uint64_t ts2 = wall_clock64();
  if (stats_tile >= 0 && stats_tile < RT_STATS_TILES && lane == 0) {
    g_tile_stats[stats_tile][0] = (uint32_t)(ts1 - ts0);
    g_tile_stats[stats_tile][1] = (uint32_t)(ts2 - ts1);
    g_tile_stats[stats_tile][2] = (uint32_t)mx | ((uint32_t)rounds << 8);
    g_tile_stats[stats_tile][3] = (uint32_t)sm;
  }
#endif
  Col C = {0.0, 0.0, 0.0};
  for (int h = nh - 1; h >= 0; --h) {
    const Col L = {hC[h][0], hC[h][1], hC[h][2]};
    const double w = hW[h];
    C = (h == nh - 1 && !last_spawned) ? L : cadd<FC>(intensify<FC>(L, 1.0 - w), intensify<FC>(C, w));   // :278-279
  }
  return C;
}

__device__ __forceinline__ DS make_ds(const RtDevScene& s) {
  DS d;
  d.objects = as_const(s.objects);
  d.trav = as_const(s.trav);
  d.n_trav = s.n_trav;
  d.strav = as_const(s.strav);
  d.n_strav = s.n_strav;
  d.nodes = as_const(s.nodes);
  d.leaves = as_const(s.leaves);
  d.prog = as_const(s.prog);
  d.lights = as_const(s.lights);
  d.textures = as_const(s.textures);
  d.texels = s.texels;
  d.n_objects = s.n_objects;
  d.n_lights = s.n_lights;
  d.shadow_early_out = s.shadow_early_out;
  return d;
}

// PerspectiveCamera::create_ray (camera.rs:65-74)
__device__ __forceinline__ void camera_ray(const RtCamera& cam, double x, double y, V3* ro, V3* rd) {
  double sx = ((x / cam.width) - 0.5) * cam.aspect;
  double sy = (cam.height - 1.0 - y) / cam.height - 0.5;
  *rd = add(add(ld3(cam.direction), scale(ld3(cam.right), sx)), scale(ld3(cam.up), sy));
  *ro = ld3(cam.center);
}

// Output rows r = 0 .. n_rows-1 of a band layout: r -> full-frame row
//   y = y_first + (r / band_rows) * band_pitch + r % band_rows
// (a contiguous tile [y0, y1) is one band; the cyclic multi-GPU layout deals bands of
// band_rows rows with pitch world * band_rows).  Workgroup = 16x16 output pixels, wave = 8x8.
// Waves per SIMD (VGPR budget 512 / N) per instantiation: reflection-only scenes (REFR = false)
// run 5 (<= 102 VGPRs, 96 used, 6 spilled).  Round 1 chose 7 (72 VGPRs, ~58 spilled) from A/B
// runs that synchronised after every launch; with launches back to back (sustained clocks,
// tools/ab_interleaved.py --burst) 5 is 1-3 % faster than 7 and cuts the launch's HBM traffic 9x
// (2.30 -> 0.245 GB: the spills went to scratch), 6 is 5 % slower, 8 spills and is 1.7x slower
// (profiles/r02o_waves_sustained.txt, r02q_ab.txt, r02r_ab.txt).  Refraction scenes with ray
// trees keep 4 (128 VGPRs; 3 is equal, 5 is 1.5 % slower, profiles/r02s_ab.txt).
// Kernel modes (RT_MODE_*): the reflection-only megakernel; refraction scenes whose rays form
// chains (RtDevScene::ray_chains: frames are (A, w) only, no pending-reflection state); refraction
// scenes with ray trees.
#define RT_MODE_REFL 0
#define RT_MODE_CHAIN 1
#define RT_MODE_TREE 2
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 4
#endif
#ifndef RT_WAVES_PER_EU_NOREFR
#define RT_WAVES_PER_EU_NOREFR 5
#endif
// The chain kernel at 4 waves/SIMD keeps every VGPR in registers (115) and 5 stack frames in LDS:
// anim120 moves 48.8 MB of HBM per 1080p frame (27 MB written, 3.3x the frame) at 9 201 Mrays/s.
// At 5 waves/SIMD it spills 27 VGPRs inside the traversal loops and moves 481.7 MB per frame (317 MB
// written) for 9 680 Mrays/s (+5 %); 5 waves without the shared sphere terms (14 spills) 216 MB at
// 8 814 (profiles/r03k_anim_variants.txt).  The traffic budget wins over 5 %, as for the megakernel.
#ifndef RT_WAVES_PER_EU_CHAIN
#define RT_WAVES_PER_EU_CHAIN 4
#endif
#define RT_WAVES(REFR) ((REFR) ? RT_WAVES_PER_EU : RT_WAVES_PER_EU_NOREFR)
#define RT_WAVES_MODE(M) ((M) == RT_MODE_REFL ? RT_WAVES_PER_EU_NOREFR : (M) == RT_MODE_CHAIN ? RT_WAVES_PER_EU_CHAIN : RT_WAVES_PER_EU)
// Workgroup = one wave of 8x8 pixels: measured 3-5 % faster than 2x2-wave workgroups (round 1).
constexpr int RT_WG_THREADS = 64;
constexpr int RT_TILE_W = 8, RT_TILE_H = 8;
#ifdef RT_DIAG_LDS_SCENE
#define RT_ROWS_WG_THREADS 256
#else
#define RT_ROWS_WG_THREADS RT_WG_THREADS
#endif
template <int MODE, bool F64, bool CAL = false, bool FC = false>
__global__ __launch_bounds__(RT_ROWS_WG_THREADS) __attribute__((amdgpu_waves_per_eu(RT_WAVES_MODE(MODE)))) void render_rows_kernel(RtDevScene S, int y_first, int band_rows, int band_pitch,
                                                          int n_rows, int max_depth, uint8_t* __restrict__ out,
                                                          size_t stride, const int32_t* __restrict__ order,
                                                          uint32_t* __restrict__ cost, int rgb) {
  constexpr bool REFR = MODE != RT_MODE_REFL, CHAIN = MODE == RT_MODE_CHAIN;
#ifdef RT_DIAG_LDS                       // diagnostic builds only: cap occupancy with an LDS pad
  __shared__ volatile char rt_pad[RT_DIAG_LDS];
  if (threadIdx.x == 0) rt_pad[0] = 0;
#endif
  const int lane = threadIdx.x & 63;
#ifdef RT_DIAG_LDS_SCENE
  // Diagnostic A/B (the north star's "node arrays staged in LDS"): 4 waves per workgroup share one
  // LDS copy of the scene tables (objects .. texture headers); every scene read below is then an LDS
  // read (ds_read, the same address on every lane) instead of a scalar load.
  constexpr int WPB = 4;
  const unsigned wave = threadIdx.x >> 6, entry = blockIdx.x * WPB + wave;
  __shared__ __attribute__((aligned(16))) uint8_t s_scene[RT_DIAG_LDS_SCENE];
  const uint8_t* b0 = (const uint8_t*)S.objects;
  const size_t nbytes = (size_t)(S.texels - b0);
  for (size_t q = threadIdx.x * 16; q < nbytes && q + 16 <= RT_DIAG_LDS_SCENE; q += WPB * 64 * 16)
    *(uint4*)&s_scene[q] = *(const uint4*)&b0[q];
  __syncthreads();
  const unsigned tile = CAL || !order ? entry : (unsigned)order[entry];
#else
  // Tile dispatch order (see launch_bands): `order` lists the tiles most expensive first, as
  // measured on a calibration launch that stored each tile's wave time in `cost`.
  // CAL (the calibration instantiation) is the only one that carries the timing code.
  const unsigned tile = CAL || !order ? blockIdx.x : (unsigned)order[blockIdx.x];
#endif
#ifdef RT_DIAG_HOT_TILES                 // diagnostic A/B builds only: issue priority for the costliest tiles
  if (!CAL && order && blockIdx.x < RT_DIAG_HOT_TILES) __builtin_amdgcn_s_setprio(3);
#endif
  [[maybe_unused]] uint64_t t_start = 0;
  if constexpr (CAL) t_start = wall_clock64();
  const unsigned tiles_x = (unsigned)(S.width + RT_TILE_W - 1) / RT_TILE_W;
  const int bx = (int)(tile % tiles_x), by = (int)(tile / tiles_x);
  const int x = bx * RT_TILE_W + (lane & 7);
  const int r = by * RT_TILE_H + (lane >> 3);
  if (x >= S.width || r >= n_rows) return;
  const int y = y_first + (r / band_rows) * band_pitch + r % band_rows;
  if (y >= S.height) return;
  V3 ro, rd;
  PROF_T0(p5);
  camera_ray(S.cam, (double)x, (double)y, &ro, &rd);                       // get_pixel(x as f64, y as f64)
#if RT_LDS_FRAMES > 0
  constexpr int KLR = MODE == RT_MODE_TREE ? RT_LDS_RFRAMES : 0;
  constexpr int KL = CHAIN ? RT_LDS_FRAMES_CHAIN : RT_LDS_FRAMES;
#ifdef RT_DIAG_LDS_SCENE
  __shared__ double s_frames[WPB][(KL * 4 + KLR * 7) * 64];
  lds_f64* lf = (lds_f64*)&s_frames[wave][lane];
  DS D = make_ds(S);
  {
    CAS uint8_t* L0 = (CAS uint8_t*)s_scene;
    auto lds = [&](const void* p) { return L0 + ((const uint8_t*)p - b0); };
    D.objects = (cptr<RtObject>)lds(S.objects);
    D.trav = (cptr<RtTrav>)lds(S.trav);
    D.strav = (cptr<RtTrav>)lds(S.strav);
    D.nodes = (cptr<RtNode>)lds(S.nodes);
    D.leaves = (cptr<RtLeaf>)lds(S.leaves);
    D.prog = (cptr<RtProg>)lds(S.prog);
    D.lights = (cptr<RtLight>)lds(S.lights);
    D.textures = (cptr<RtTexture>)lds(S.textures);
  }
  const Col c = trace<REFR, NoRec, KL, FC, KLR, CHAIN>(D, ro, rd, max_depth, nullptr, lf);
#else
  __shared__ double s_frames[(KL * 4 + KLR * 7) * 64];   // frame stack, see trace()
  lds_f64* lf = (lds_f64*)&s_frames[lane];
  const Col c = trace<REFR, NoRec, KL, FC, KLR, CHAIN>(make_ds(S), ro, rd, max_depth, nullptr, lf);
#endif
#else
  const Col c = trace<REFR, NoRec, 0, FC, 0, CHAIN>(make_ds(S), ro, rd, max_depth);
#endif
  PROF_ADD(5, p5);
  uint8_t* row = out + (size_t)r * stride;
  if constexpr (F64) {
    double* o = (double*)row + (size_t)x * 4;
    o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = 1.0;                        // alpha is 1 after any colour op
  } else if (rgb) {                                                        // packed RGB8 (band gathers)
    uint8_t* o = row + (size_t)x * 3;
    o[0] = (uint8_t)to_u8(c.r); o[1] = (uint8_t)to_u8(c.g); o[2] = (uint8_t)to_u8(c.b);
  } else {
    ((uint32_t*)row)[x] = to_u8(c.r) | (to_u8(c.g) << 8) | (to_u8(c.b) << 16) | (255u << 24);
  }
  if constexpr (CAL)
    if (threadIdx.x == 0) cost[tile] = (uint32_t)(wall_clock64() - t_start);   // vector store
}

// The deferred-shadow kernel for scenes without a transparent object (REFR = false), used for
// launches of few tiles (a multi-GPU rank's share), whose time is set by their costliest tiles:
// one wave per 8x8 tile as above, every tile on the deferred path (trace_deferred), and the
// costliest tiles split over P = 2, 4 or 8 waves: wave `part` renders pixels
// [part * 64/P, (part + 1) * 64/P) of the tile on its first 64/P lanes and its other lanes only
// trace shadow rays (phase 2), so a costly tile's shadow work spreads over P x 64 lanes and its
// latency -- the launch's tail -- shrinks.  Order entry: tile | part << 20 | log2(P) << 24 (built
// by launch_bands after the calibration launch).  A kernel of its own: the megakernel path and
// this one in ONE kernel measured 3.4x slower than either (profiles/r02g_ab.txt: both paths' code
// hot on one CU at once).
#ifndef RT_WAVES_PER_EU_DEFERRED
#define RT_WAVES_PER_EU_DEFERRED 7
#endif
#ifdef RT_DIAG_ENTRY_TIMES                // diagnostic build only: per dispatched entry, start / end ticks
#define RT_ENTRY_TIMES_MAX (1 << 20)
__device__ unsigned long long g_entry_times[RT_ENTRY_TIMES_MAX][2];
__device__ unsigned g_diag_hot;             // entries below this index run at issue priority 3
#endif
template <bool F64, bool CAL = false, bool FC = false, bool REFR = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU_DEFERRED))) void
render_rows_deferred_kernel(RtDevScene S, int y_first, int band_rows, int band_pitch, int n_rows, int max_depth,
                            uint8_t* __restrict__ out, size_t stride, const int32_t* __restrict__ order,
                            uint32_t* __restrict__ cost, int rgb) {
  __shared__ ShadowWin win;
  const int lane = threadIdx.x & 63;
#ifdef RT_DIAG_ENTRY_TIMES
  const unsigned long long et0 = wall_clock64();
  if (!CAL && order && blockIdx.x < g_diag_hot) __builtin_amdgcn_s_setprio(3);
#endif
  const uint32_t e = CAL || !order ? blockIdx.x : (uint32_t)order[blockIdx.x];
  const unsigned tile = e & RT_SPLIT_TILE_MASK;
  const int lp = (int)((e >> 24) & 7u), per = 64 >> lp;
  const int pix = (int)((e >> 20) & 15u) * per + lane;
  [[maybe_unused]] uint64_t t_start = 0;
  if constexpr (CAL) t_start = wall_clock64();
  const unsigned tiles_x = (unsigned)(S.width + 7) / 8;
  const int x = (int)(tile % tiles_x) * 8 + (pix & 7);
  const int r = (int)(tile / tiles_x) * 8 + (pix >> 3);
  int y = 0;
  bool valid = lane < per && x < S.width && r < n_rows;
  if (valid) {
    y = y_first + (r / band_rows) * band_pitch + r % band_rows;
    valid = y < S.height;
  }
  V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
  if (valid) camera_ray(S.cam, (double)x, (double)y, &ro, &rd);             // get_pixel(x as f64, y as f64)
  const Col c = trace_deferred<RT_MAX_DEPTH_CAP + 1, FC, REFR>(make_ds(S), ro, rd, max_depth, valid, &win, CAL ? (int)tile : -1);
  if (valid) {
    uint8_t* row = out + (size_t)r * stride;
    if constexpr (F64) {
      double* o = (double*)row + (size_t)x * 4;
      o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = 1.0;
    } else if (rgb) {
      uint8_t* o = row + (size_t)x * 3;
      o[0] = (uint8_t)to_u8(c.r); o[1] = (uint8_t)to_u8(c.g); o[2] = (uint8_t)to_u8(c.b);
    } else {
      ((uint32_t*)row)[x] = to_u8(c.r) | (to_u8(c.g) << 8) | (to_u8(c.b) << 16) | (255u << 24);
    }
  }
  if constexpr (CAL)
    if (lane == 0) cost[tile] = (uint32_t)(wall_clock64() - t_start);
#ifdef RT_DIAG_ENTRY_TIMES
  if (!CAL && lane == 0 && blockIdx.x < RT_ENTRY_TIMES_MAX) {
    g_entry_times[blockIdx.x][0] = et0;
    g_entry_times[blockIdx.x][1] = wall_clock64();
  }
#endif
}

// ====================================================================== wavefront path
// get_ray_color (raytracer.rs:132-287) launch-wide, one bounce level per pass: level d holds every
// ray of recursion depth d of the launch, densely, one lane per ray.  Per level:
//   wf_trace_kernel  nearest hit, shadow rays, shading, the inside / refraction / TIR / reflection
//                    decisions of trace() (the same operations in the same order); the rays a hit
//                    spawns are appended to level d + 1 (one ballot + one atomic per wave), each with a
//                    coherence key (direction octant, Morton code of its origin); the hit record (L,
//                    the two weights, the children's slots) stays at the ray's slot;
//   sort             level d + 1's slots by key (rocPRIM radix sort of (key, slot) pairs): a wave of
//                    the next pass then traces rays that start close together in similar directions,
//                    so the wave-coherent traversal walks fewer objects (the megakernel's waves walk the
//                    union of what their lanes' scattered secondary rays need);
//   wf_fold_kernel   after every level is traced, from the deepest level up: a ray's colour from its
//                    hit record and its children's colours (already folded into their L slots):
//                      refraction child: comb = in_range(L.intensify(1 - t) + C_t.intensify(t)),
//                      then a reflection child: in_range(comb.intensify(1 - rp) + C_r.intensify(rp)),
//                    exactly the post-order of raytracer.rs:256-279 (trace()'s frame fold).  Level 0's
//                    fold writes the pixels.
// Lanes whose pixel's tree ended early no longer idle in its wave (the megakernel's per-lane tree
// walk keeps a wave alive for its deepest tree): every pass starts with every lane on a live ray, and
// every pass is one workgroup per 64 rays, so the hardware dispatcher balances uneven rays.  The
// host reads each level's count before launching it (one synchronisation per level: this path is
// for heavy, incoherent launches).  Levels >= 1 hold RT_OPT_WAVEFRONT_CAP % of the pixel slots; a
// ray that finds its level full marks its pixel, and wf_fixup_kernel re-renders marked pixels with
// trace() (same bits).
struct WfArena {
  uint8_t* base;          // level tables (wf_level)
  uint32_t* count;        // count[d]: rays appended to level d (d >= 1); count[RT_MAX_DEPTH_CAP + 2]: any overflow
  uint8_t* ovf;           // per pixel slot: its tree overflowed a level
  const uint32_t* perm;   // the level being traced: slot of its i-th ray in key order (null: slot order)
  uint32_t slots, cap;    // level 0 = the pixel slots (8x8 tiles x 64), levels >= 1: cap rays each
  double klo[3], kscale[3];   // origin -> 9-bit cell per axis for the coherence keys
};
struct WfLevel {
  double *ox, *oy, *oz, *dx, *dy, *dz;   // levels >= 1: the ray
  double *Lr, *Lg, *Lb, *wt, *wr;        // hit record: L (then the folded colour), refraction / reflection weights
  int32_t *pix, *ct, *cr;                // pixel slot (levels >= 1), children's slots in level d + 1 (-1: none)
  uint32_t *key, *val;                   // levels >= 1: coherence key and slot (the sort's input pairs)
  int32_t* par;                          // levels >= 1: the object whose hit spawned the ray
};
constexpr size_t RT_WF_BYTES0 = 5 * 8 + 2 * 4, RT_WF_BYTES = 11 * 8 + 6 * 4;
__host__ __device__ __forceinline__ WfLevel wf_level(const WfArena& A, int d) {
  WfLevel v;
  const size_t len = d == 0 ? A.slots : A.cap;
  double* f = (double*)(A.base + (d == 0 ? 0 : (size_t)A.slots * RT_WF_BYTES0 + (size_t)(d - 1) * A.cap * RT_WF_BYTES));
  if (d == 0) {
    v.ox = v.oy = v.oz = v.dx = v.dy = v.dz = nullptr;
    v.Lr = f; v.Lg = f + len; v.Lb = f + 2 * len; v.wt = f + 3 * len; v.wr = f + 4 * len;
    int32_t* q = (int32_t*)(f + 5 * len);
    v.pix = nullptr; v.ct = q; v.cr = q + len;
    v.key = v.val = nullptr;
    v.par = nullptr;
  } else {
    v.ox = f; v.oy = f + len; v.oz = f + 2 * len; v.dx = f + 3 * len; v.dy = f + 4 * len; v.dz = f + 5 * len;
    v.Lr = f + 6 * len; v.Lg = f + 7 * len; v.Lb = f + 8 * len; v.wt = f + 9 * len; v.wr = f + 10 * len;
    int32_t* q = (int32_t*)(f + 11 * len);
    v.pix = q; v.ct = q + len; v.cr = q + 2 * len;
    v.key = (uint32_t*)(q + 3 * len); v.val = (uint32_t*)(q + 4 * len);
    v.par = q + 5 * len;
  }
  return v;
}
// pixel slot -> (x, output row r); false outside the launch's rows / frame
__device__ __forceinline__ bool wf_pixel(const RtDevScene& S, uint32_t slot, int y_first, int band_rows, int band_pitch,
                                         int n_rows, int* x, int* r, int* y) {
  const unsigned tiles_x = (unsigned)(S.width + 7) / 8, tile = slot >> 6, l = slot & 63;
  *x = (int)(tile % tiles_x) * 8 + (int)(l & 7);
  *r = (int)(tile / tiles_x) * 8 + (int)(l >> 3);
  if (*x >= S.width || *r >= n_rows) return false;
  *y = y_first + (*r / band_rows) * band_pitch + *r % band_rows;
  return *y < S.height;
}
// coherence key of a ray: direction octant (3 bits) above the 27-bit Morton code of its origin's
// cell (9 bits per axis over the scene's bounded extent, clamped).  Only the processing order
// depends on it, never a value.
__device__ __forceinline__ uint32_t wf_spread9(uint32_t v) {            // 9 bits -> every third bit
  v &= 511u;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}
__device__ __forceinline__ uint32_t wf_key(const WfArena& A, V3 o, V3 d) {
  auto cell = [](double x, double lo, double sc) -> uint32_t {
    const double c = (x - lo) * sc;
    return c > 0.0 ? (c < 511.0 ? (uint32_t)c : 511u) : 0u;           // NaN -> 0
  };
  const uint32_t oct = (d.x < 0.0 ? 1u : 0u) | (d.y < 0.0 ? 2u : 0u) | (d.z < 0.0 ? 4u : 0u);
  return (oct << 27) | wf_spread9(cell(o.x, A.klo[0], A.kscale[0])) | (wf_spread9(cell(o.y, A.klo[1], A.kscale[1])) << 1) |
         (wf_spread9(cell(o.z, A.klo[2], A.kscale[2])) << 2);
}

// One ray of trace()'s loop body: nearest hit, the light loop (shadow rays first, then the shading
// inputs), the inside test and the refraction / reflection decisions (raytracer.rs:141-280).
// NH(&t) gives the nearest hit (object, distance), SH(k, p, sdir, dist) light k's shadow
// transparency: the traversals themselves (wf_ray) or the pair path's folded results (wfp_shade).
template <bool REFR, bool FC, class NH, class SH>
__device__ __forceinline__ void wf_ray_core(const DS& S, V3 ro, V3 rd, int depth, int max_depth, NH&& nh, SH&& sh,
                                            Col* Lo, double* wt, double* wr, bool* ch_t, bool* ch_r, V3* po, V3* dt,
                                            V3* dr) {
  *ch_t = *ch_r = false;
  *Lo = {0.0, 0.0, 0.0};
  *wt = *wr = 0.0;
  double t_hit;
  const int oi = nh(&t_hit);
  if (oi < 0) return;                                                   // Color::BLACK (:152-160)
  const V3 p = add(ro, scale(rd, t_hit));                               // :162
  V3 nrm = {0.0, 0.0, 0.0};
  Col c = {0.0, 0.0, 0.0}, L = {0.0, 0.0, 0.0};
  double transp = 0.0, refl = 0.0;
  bool have_shading = false;
#pragma unroll 1
  for (int k = 0; k < S.n_lights; ++k) {                                // :175-228, as trace()
    cptr<RtLight> lt = &S.lights[k];
    const V3 lv = sub(ld3(lt->p), p);
    double ll, ill;
    len_inv(lv, &ll, &ill);
    const V3 sdir = scale(lv, ill);
    const double t = sh(k, p, sdir, ll);
    if (!have_shading) {
      shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);
      L = cmul<FC>(c, in_range<FC>(0.6, 0.6, 0.6));
      have_shading = true;
    }
    if (t == 0.0) continue;
    double ang = rt_acos(dot(sdir, nrm) / (len(sdir) * len(nrm)));
    if (ang >= PI_D / 2.0) ang = PI_D - ang;
    const double inten = (ang < (PI_D / 2.0) && ang >= 0.0) ? 1.0 - (ang / (PI_D / 2.0)) : 0.0;
    const Col lc = intensify<FC>(intensify<FC>(Col{lt->col[0], lt->col[1], lt->col[2]}, inten), t);
    L = cadd<FC>(L, cmul<FC>(c, lc));
  }
  if (!have_shading) {
    shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);
    L = cmul<FC>(c, in_range<FC>(0.6, 0.6, 0.6));
  }
  bool inside = false;                                                  // :230-235
  if (depth < max_depth && (refl != 0.0 || (REFR && transp != 0.0))) {
    const V3 nd = scale(rd, -1.0);
    inside = inside_test(dot(nd, nrm) / (len(nd) * len(nrm)));
  }
  const V3 n2 = inside ? scale(nrm, -1.0) : nrm;
  const double r1 = inside ? 1.45 : 1.0, r2 = inside ? 1.0 : 1.45;
  bool tir = false;
  V3 tdir = {0.0, 0.0, 0.0};
  const bool do_refr = REFR && depth < max_depth && transp != 0.0;     // :242
  if (do_refr) tdir = refract_dir(rd, n2, r1 / r2, &tir);
  const double rp = tir ? refl + (1.0 - refl) * transp : refl;         // :261-265
  const bool do_refl = depth < max_depth && rp != 0.0 && (!inside || tir);   // :267
  *Lo = L;
  *wt = transp;
  *wr = rp;
  *ch_t = do_refr && !tir;
  *ch_r = do_refl;
  *po = p;
  *dt = tdir;
  if (do_refl) *dr = reflect_dir(rd, n2);
}

template <bool REFR, bool FC>
__device__ __forceinline__ void wf_ray(const DS& S, V3 ro, V3 rd, int depth, int max_depth, Col* Lo, double* wt,
                                       double* wr, bool* ch_t, bool* ch_r, V3* po, V3* dt, V3* dr, int* hit_obj) {
  constexpr bool SHARE = REFR && RT_SPHERE_SHARE, OBB = !REFR;
  wf_ray_core<REFR, FC>(
      S, ro, rd, depth, max_depth,
      [&](double* t) { return *hit_obj = nearest_hit<SHARE, OBB>(S, ro, rd, t, depth == 0 ? 0 : 1); },
      [&](int, V3 p, V3 sdir, double ll) { return shadow_transparency<SHARE, OBB>(S, p, sdir, ll); }, Lo, wt, wr, ch_t,
      ch_r, po, dt, dr);
}

// The rays a wave's hits spawn, appended to level d + 1 (one ballot per kind, ONE atomic per
// wave: the wave's refraction children, then its reflection children, in lane order), and the hit
// record at the ray's slot j.
__device__ __forceinline__ void wf_append(const WfArena& A, const WfLevel& lv, int d, int lane, bool live, uint32_t j,
                                          int32_t pix, Col L, double wt, double wr, bool ch_t, bool ch_r, V3 p, V3 dt,
                                          V3 dr, int32_t par = -1) {
  int32_t ct = -1, cr = -1;
  const uint64_t bt = __ballot(ch_t), br = __ballot(ch_r);
  const uint32_t nt = (uint32_t)__popcll(bt), nr = (uint32_t)__popcll(br);
  if (nt + nr) {                                             // wave-uniform: d < max_depth here
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t b0 = 0;
    if (lane == 0) b0 = atomicAdd(&A.count[d + 1], nt + nr);
    b0 = (uint32_t)__shfl((int)b0, 0);
    const WfLevel nx = wf_level(A, d + 1);
    const uint32_t st = b0 + (uint32_t)__popcll(bt & below), sr = b0 + nt + (uint32_t)__popcll(br & below);
    bool ovf = false;
    if (ch_t) {
      if (st < A.cap) {
        nx.ox[st] = p.x; nx.oy[st] = p.y; nx.oz[st] = p.z; nx.dx[st] = dt.x; nx.dy[st] = dt.y; nx.dz[st] = dt.z;
        nx.pix[st] = pix; nx.key[st] = wf_key(A, p, dt); nx.val[st] = st; nx.par[st] = par;
        ct = (int32_t)st;
      } else ovf = true;
    }
    if (ch_r) {
      if (sr < A.cap) {
        nx.ox[sr] = p.x; nx.oy[sr] = p.y; nx.oz[sr] = p.z; nx.dx[sr] = dr.x; nx.dy[sr] = dr.y; nx.dz[sr] = dr.z;
        nx.pix[sr] = pix; nx.key[sr] = wf_key(A, p, dr); nx.val[sr] = sr; nx.par[sr] = par;
        cr = (int32_t)sr;
      } else ovf = true;
    }
    if (ovf) {                                                // this pixel is re-rendered by wf_fixup_kernel
      A.ovf[pix] = 1;
      A.count[RT_MAX_DEPTH_CAP + 2] = 1;
    }
  }
  if (live) {
    lv.Lr[j] = L.r; lv.Lg[j] = L.g; lv.Lb[j] = L.b; lv.wt[j] = wt; lv.wr[j] = wr;
    lv.ct[j] = ct; lv.cr[j] = cr;
  }
}

#ifndef RT_WAVES_PER_EU_WF
#define RT_WAVES_PER_EU_WF 5
#endif
// One workgroup (wave) per 64 rays of level d (n of them): level 0 = the pixel slots in tile order,
// levels >= 1 in key order (A.perm).
template <bool REFR, bool FC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU_WF))) void wf_trace_kernel(
    RtDevScene S, WfArena A, int d, uint32_t n, int y_first, int band_rows, int band_pitch, int n_rows, int max_depth) {
  const int lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 64u + (uint32_t)lane;
  bool live = i < n;
  const WfLevel lv = wf_level(A, d);
  V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
  uint32_t j = i;                                            // the ray's slot in its level
  int32_t pix = (int32_t)i;
  if (d == 0) {
    int x, r, y;
    live = live && wf_pixel(S, i, y_first, band_rows, band_pitch, n_rows, &x, &r, &y);
    if (live) camera_ray(S.cam, (double)x, (double)y, &ro, &rd);          // get_pixel(x as f64, y as f64)
  } else if (live) {
    j = A.perm ? A.perm[i] : i;
    ro = {lv.ox[j], lv.oy[j], lv.oz[j]};
    rd = {lv.dx[j], lv.dy[j], lv.dz[j]};
    pix = lv.pix[j];
  }
  Col L = {0.0, 0.0, 0.0};
  double wt = 0.0, wr = 0.0;
  bool ch_t = false, ch_r = false;
  V3 p = {0.0, 0.0, 0.0}, dt = {0.0, 0.0, 0.0}, dr = {0.0, 0.0, 0.0};
  int oi = -1;
  if (live) wf_ray<REFR, FC>(make_ds(S), ro, rd, d, max_depth, &L, &wt, &wr, &ch_t, &ch_r, &p, &dt, &dr, &oi);
  wf_append(A, lv, d, lane, live, j, pix, L, wt, wr, ch_t, ch_r, p, dt, dr, oi);
}

template <bool F64, bool FC>
__global__ __launch_bounds__(256) void wf_fold_kernel(RtDevScene S, WfArena A, int d, uint32_t n, int y_first,
                                                      int band_rows, int band_pitch, int n_rows,
                                                      uint8_t* __restrict__ out, size_t stride, int rgb) {
  const WfLevel lv = wf_level(A, d);
  const WfLevel ch = wf_level(A, d + 1);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int x = 0, r = 0, y = 0;
    if (d == 0 && (!wf_pixel(S, i, y_first, band_rows, band_pitch, n_rows, &x, &r, &y) || A.ovf[i])) continue;
    const Col L = {lv.Lr[i], lv.Lg[i], lv.Lb[i]};
    const int32_t ct = lv.ct[i], cr = lv.cr[i];
    Col C = L;
    if (ct >= 0) {                                             // refraction, then a pending reflection
      const double t = lv.wt[i];
      C = cadd<FC>(intensify<FC>(L, 1.0 - t), intensify<FC>(Col{ch.Lr[ct], ch.Lg[ct], ch.Lb[ct]}, t));
    }
    if (cr >= 0) {
      const double w = lv.wr[i];
      C = cadd<FC>(intensify<FC>(C, 1.0 - w), intensify<FC>(Col{ch.Lr[cr], ch.Lg[cr], ch.Lb[cr]}, w));
    }
    if (d > 0) {
      lv.Lr[i] = C.r; lv.Lg[i] = C.g; lv.Lb[i] = C.b;
      continue;
    }
    uint8_t* row = out + (size_t)r * stride;
    if constexpr (F64) {
      double* o = (double*)row + (size_t)x * 4;
      o[0] = C.r; o[1] = C.g; o[2] = C.b; o[3] = 1.0;
    } else if (rgb) {
      uint8_t* o = row + (size_t)x * 3;
      o[0] = (uint8_t)to_u8(C.r); o[1] = (uint8_t)to_u8(C.g); o[2] = (uint8_t)to_u8(C.b);
    } else {
      ((uint32_t*)row)[x] = to_u8(C.r) | (to_u8(C.g) << 8) | (to_u8(C.b) << 16) | (255u << 24);
    }
  }
}

// Pixels whose tree overflowed a level: the per-lane megakernel trace (same bits).  Returns at once
// when no level overflowed (one uniform load).
template <bool REFR, bool F64, bool FC>
__global__ __launch_bounds__(64) void wf_fixup_kernel(RtDevScene S, WfArena A, int y_first, int band_rows,
                                                      int band_pitch, int n_rows, int max_depth,
                                                      uint8_t* __restrict__ out, size_t stride, int rgb) {
  if (A.count[RT_MAX_DEPTH_CAP + 2] == 0) return;
  for (uint32_t i = blockIdx.x * 64 + threadIdx.x; i < A.slots; i += gridDim.x * 64) {
    int x, r, y;
    if (!A.ovf[i] || !wf_pixel(S, i, y_first, band_rows, band_pitch, n_rows, &x, &r, &y)) continue;
    V3 ro, rd;
    camera_ray(S.cam, (double)x, (double)y, &ro, &rd);
    const Col C = trace<REFR, NoRec, 0, FC>(make_ds(S), ro, rd, max_depth);
    uint8_t* row = out + (size_t)r * stride;
    if constexpr (F64) {
      double* o = (double*)row + (size_t)x * 4;
      o[0] = C.r; o[1] = C.g; o[2] = C.b; o[3] = 1.0;
    } else if (rgb) {
      uint8_t* o = row + (size_t)x * 3;
      o[0] = (uint8_t)to_u8(C.r); o[1] = (uint8_t)to_u8(C.g); o[2] = (uint8_t)to_u8(C.b);
    } else {
      ((uint32_t*)row)[x] = to_u8(C.r) | (to_u8(C.g) << 8) | (to_u8(C.b) << 16) | (255u << 24);
    }
  }
}

// ---------------------------------------------------------------- wavefront pair path
// A level's rays are incoherent after a few bounces through scenes of many objects (fractal.scene:
// 171 objects, glass spheres in hollow CSG cubes).  A wave that walks the hierarchy for 64 scattered
// rays visits the union of their paths: on fractal.scene only 14 % / 22 % of the lanes are active in
// a secondary / shadow leaf evaluation, and every level's pass takes as long as a wave's walk over
// most of the scene (0.6-2 ms even for 25 000 rays).  The pair path splits the traversal into
// (ray, object) work items and evaluates them object by object:
//   wfp_cand_kernel<false>   per ray: the hierarchy walk with box tests only (no leaf), emitting a
//                            pair (object, ray) for every object box the ray meets (through a per-wave
//                            LDS buffer, one atomic per RT_WFP_BUF pairs);
//   sort                     the pairs by object (rocPRIM radix sort), so a wave evaluates ONE object
//                            (scalar loads of its leaves, every lane busy) for 64 different rays;
//   wfp_near_eval_kernel     per pair: the object's nearest accepted distance (leaf tests, CSG filters:
//                            nearest_hit's object body); atomicMin of its bits into the ray's best;
//   wfp_near_tie_kernel      per pair at the ray's best distance: atomicMin of the object index.  The
//                            nearest hit is the least (distance, object) -- exactly nearest_hit's
//                            draw-order first-wins rule (raytracer.rs:141-150);
//   wfp_cand_kernel<true>    per ray with a hit and per light: the shadow ray's candidate objects;
//   sort, wfp_shadow_eval    per pair: the object's filtered hits with EPS < t < dist; a hit of a
//                            zero-transparency object marks the shadow ray opaque, other hits add to
//                            its count.  RtDevScene::shadow_pow (scene.cpp) guarantees the product in
//                            draw order is then 0 or T^count, order-free (raytracer.rs:181-197);
//   wfp_shade_kernel         per ray: wf_ray_core's shading, refraction and reflection decisions with
//                            the folded results, then wf_append, as wf_trace_kernel.
// Every value is computed by the same operations as the traversals; culling stays conservative
// (the candidate walk tests boxes against the whole ray, tmax = infinity for the nearest hit).
struct WfPairs {
  uint32_t *key, *val;          // pairs as emitted: object, ray id (level slot, or slot * n_lights + light)
  uint32_t *key_s, *val_s;      // sorted by object
  double* tp;                   // nearest pass: the sorted pair's object's nearest accepted distance
  uint32_t* count;              // [0] / [1]: pairs the nearest / shadow pass emitted (may exceed cap: the host
                                //   grows the arena and runs the level again)
  uint32_t* bins;               // bucket-sort scratch (RT_BS_MAX_BINS words)
  uint32_t cap;
  unsigned long long* tmin;     // per ray of the level: nearest accepted distance (bits; +inf: none)
  int32_t* omin;                // per ray: the least object index at that distance (INT_MAX: none)
  double *px, *py, *pz;         // per ray: the hit point
  uint32_t *kcnt, *opq;         // per shadow ray: hits of transparency-T objects / of a zero-transparency one
  uint32_t *hkey, *hval, *hkey_s, *hperm;   // per ray: hit-point key, slot; sorted: the shadow / shading order
};
#ifndef RT_WFP_BUF
#define RT_WFP_BUF 512          // pairs buffered in LDS per wave before one atomic allocates their slots
#endif
constexpr unsigned long long RT_WFP_NONE = 0x7FF0000000000000ull;   // +inf
constexpr int RT_WFP_COUNT = 32;      // the pair counts' words in WfArena::count (after the level counts)
static_assert(RT_MAX_DEPTH_CAP + 3 <= RT_WFP_COUNT, "wavefront counter block");

// The object's nearest accepted distance for one ray: nearest_hit's body for one object, its best
// starting at +inf (the leaf boxes' tmax only shrinks, as share_prev requires).
__device__ __forceinline__ double wfp_object_nearest(const DS& S, int o, V3 ro, V3 rd, const CullRay& cr) {
  cptr<RtObject> O = &S.objects[o];
  const bool fin = wave_finite(ro, rd);
  double best = INFINITY;
  SphereShare shr = {0.0, 0.0, 0.0};
  const int lb = O->leaf_begin, le = lb + O->leaf_count;
  for (int l = lb; l < le; ++l) {
    cptr<RtLeaf> L = &S.leaves[l];
    if (O->leaf_cull) {
      if (L->cull == RT_CULL_ALWAYS) continue;
      if (L->cull == RT_CULL_BOX && !box_may_hit(L->blo, L->bhi, cr, cull_tmax(best))) continue;
    }
    double t0 = 0.0, t1 = 0.0;
    const int n = leaf_candidates<true>(L, ro, rd, fin, &t0, &t1, RT_SPHERE_SHARE ? &shr : nullptr);
    const bool filtered = L->prog_end != L->prog_begin && !(RT_CONST_FILTER && L->filter_const && !isnan(cr.inv.x));
    if (n >= 1 && t0 > EPS && t0 < best && (!filtered || leaf_filter(S, L, add(ro, scale(rd, t0))))) best = t0;
    if (n >= 2 && t1 > EPS && t1 < best && (!filtered || leaf_filter(S, L, add(ro, scale(rd, t1))))) best = t1;
  }
  return best;
}

// Filtered hits of the object with EPS < t < dist on one shadow ray (shadow_transparency's body for
// one object); a zero-transparency object stops at its first.
__device__ __forceinline__ uint32_t wfp_object_shadow(const DS& S, int o, V3 p, V3 dir, double dist, const CullRay& cr) {
  cptr<RtObject> O = &S.objects[o];
  const bool fin = wave_finite(p, dir);
  const double tmax = cull_tmax(dist);
  const bool zero = O->transparency == 0.0;
  uint32_t cnt = 0;
  SphereShare shr = {0.0, 0.0, 0.0};
  const int lb = O->leaf_begin, le = lb + O->leaf_count;
  for (int l = lb; l < le; ++l) {
    cptr<RtLeaf> L = &S.leaves[l];
    if (O->leaf_cull) {
      if (L->cull == RT_CULL_ALWAYS) continue;
      if (L->cull == RT_CULL_BOX && !box_may_hit(L->blo, L->bhi, cr, tmax)) continue;
    }
    double t0 = 0.0, t1 = 0.0;
    const int n = leaf_candidates<true>(L, p, dir, fin, &t0, &t1, RT_SPHERE_SHARE ? &shr : nullptr);
    const bool filtered = L->prog_end != L->prog_begin && !(RT_CONST_FILTER && L->filter_const && !isnan(cr.inv.x));
    if (n >= 1 && t0 > EPS && t0 < dist && (!filtered || leaf_filter(S, L, add(p, scale(dir, t0))))) {
      ++cnt;
      if (zero) return cnt;
    }
    if (n >= 2 && t1 > EPS && t1 < dist && (!filtered || leaf_filter(S, L, add(p, scale(dir, t1))))) {
      ++cnt;
      if (zero) return cnt;
    }
  }
  return cnt;
}

// Ray of slot j of level d (level 0: the pixel slot's camera ray).
__device__ __forceinline__ bool wf_get_ray(const RtDevScene& S, const WfLevel& lv, int d, uint32_t j, int y_first,
                                           int band_rows, int band_pitch, int n_rows, V3* ro, V3* rd) {
  if (d == 0) {
    int x, r, y;
    if (!wf_pixel(S, j, y_first, band_rows, band_pitch, n_rows, &x, &r, &y)) return false;
    camera_ray(S.cam, (double)x, (double)y, ro, rd);
    return true;
  }
  *ro = {lv.ox[j], lv.oy[j], lv.oz[j]};
  *rd = {lv.dx[j], lv.dy[j], lv.dz[j]};
  return true;
}

// One wave per 64 rays of level d (in key order).  SHADOW = false: every object whose box the ray
// meets; true: per light, every object whose box the shadow segment meets (objects of transparency 1
// skipped, as shadow_transparency does).
// Each lane walks its own path through the hierarchy (per-lane vector loads of one 64-byte RtTrav
// record per step, which carries the object's box and flags): a wave-uniform walk visits the union
// of its 64 rays' paths, measured 4-20 % slower here (profiles/r03m_pairs_fractal_timing.txt).
template <bool SHADOW>
__global__ __launch_bounds__(64) void wfp_cand_kernel(RtDevScene S, WfArena A, WfPairs P, int d, uint32_t n,
                                                      int y_first, int band_rows, int band_pitch, int n_rows) {
  __shared__ uint32_t sk[RT_WFP_BUF], sv[RT_WFP_BUF];
  const int lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 64u + (uint32_t)lane;
  const WfLevel lv = wf_level(A, d);
  const DS D = make_ds(S);
  bool live = i < n;
  uint32_t j = i;
  V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
  if (live) {
    j = SHADOW ? P.hperm[i] : (d > 0 && A.perm) ? A.perm[i] : i;
    if (!SHADOW) live = wf_get_ray(S, lv, d, j, y_first, band_rows, band_pitch, n_rows, &ro, &rd);
  }
  uint32_t nb = 0;                                           // wave-uniform fill of the LDS buffer
  auto flush = [&]() {
    __syncthreads();
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(P.count + (SHADOW ? 1 : 0), nb);
    base = (uint32_t)__shfl((int)base, 0);
    for (uint32_t q = (uint32_t)lane; q < nb; q += 64)
      if (base + q < P.cap) { P.key[base + q] = sk[q]; P.val[base + q] = sv[q]; }
    __syncthreads();
    nb = 0;
  };
  auto emit = [&](bool h, uint32_t ob, uint32_t id) {
    const uint64_t m = __ballot(h);
    if (!m) return;
    const uint32_t c = (uint32_t)__popcll(m);
    if (nb + c > RT_WFP_BUF) flush();
    if (h) {
      const uint32_t q = nb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      sk[q] = ob;
      sv[q] = id;
    }
    nb += c;
  };
  auto walk = [&](bool act0, V3 o, V3 dir, double tmax, uint32_t id) {
    const CullRay cr = cull_ray(o, dir);
    const RtTrav* __restrict__ TR = S.trav;
    const int nt = S.n_trav;
    int t = act0 ? 0 : nt;
    while (__ballot(t < nt)) {
      bool h = false;
      int ob = 0;
      if (t < nt) {
        const RtTrav T = TR[t];
        const bool in = box_may_hit(T.blo, T.bhi, cr, tmax);
        if (T.obj < 0) {
          t = in ? t + 1 : T.skip;
        } else {
          ++t;
          ob = T.obj;
          h = T.cull != RT_CULL_ALWAYS && !(SHADOW && T.shadow_skip) && (T.cull != RT_CULL_BOX || in);
        }
      }
      emit(h, (uint32_t)ob, id);
    }
  };
  if constexpr (!SHADOW) {
    if (i < n) { P.tmin[j] = RT_WFP_NONE; P.omin[j] = 0x7fffffff; }   // slots outside the frame too
    // A bound on the nearest hit: the object whose hit spawned the ray, evaluated first (a ray that
    // refracted into or reflects inside a closed shape meets it again).  The walk then tests boxes
    // against [0, cull_tmax(bound)] only -- conservative, as nearest_hit's running best is; the
    // parent's own pair is still emitted by the walk (its box contains the bound's point).
    double bound = INFINITY;
    if (d > 0) {
      const int32_t par = live ? lv.par[j] : -1;
      const CullRay cr = cull_ray(ro, rd);
      uint64_t todo = __ballot(live && par >= 0);
      while (todo) {                     // the children of one shading wave: mostly one parent
        const int pu = __builtin_amdgcn_readlane(par, (int)__builtin_ctzll(todo));
        const uint64_t mine = __ballot(live && par == pu);
        todo &= ~mine;
        if ((mine >> lane) & 1) bound = wfp_object_nearest(D, pu, ro, rd, cr);
      }
    }
    walk(live, ro, rd, bound < INFINITY ? cull_tmax(bound) : INFINITY, j);
  } else {
    const int32_t oi = live ? P.omin[j] : 0x7fffffff;
    const bool hit = live && oi != 0x7fffffff;
    V3 p = {0.0, 0.0, 0.0};
    if (hit) p = {P.px[j], P.py[j], P.pz[j]};                     // wfp_hit_key_kernel
    for (int k = 0; k < D.n_lights; ++k) {
      V3 sdir = {0.0, 0.0, 0.0};
      double tmax = 0.0;
      const uint32_t s = j * (uint32_t)D.n_lights + (uint32_t)k;
      if (hit) {
        cptr<RtLight> lt = &D.lights[k];
        const V3 l = sub(ld3(lt->p), p);
        double ll, ill;
        len_inv(l, &ll, &ill);
        sdir = scale(l, ill);
        tmax = cull_tmax(ll);
        P.kcnt[s] = 0;
        P.opq[s] = 0;
      }
      walk(hit, p, sdir, tmax, s);
    }
  }
  flush();
}

// One lane per sorted pair: the waves see one object (two at a run boundary): scalarised over the
// distinct objects of the wave as shade_inputs does, so every scene read is a scalar load.
__global__ __launch_bounds__(64) void wfp_near_eval_kernel(RtDevScene S, WfArena A, WfPairs P, int d, int y_first,
                                                           int band_rows, int band_pitch, int n_rows) {
  const int lane = threadIdx.x & 63;
  const uint32_t np = min(P.count[0], P.cap);               // pairs of this level's nearest pass (device)
  const WfLevel lv = wf_level(A, d);
  const DS D = make_ds(S);
  for (uint32_t base = blockIdx.x * 64u; base < np; base += gridDim.x * 64u) {   // wave-uniform bounds
    const uint32_t i = base + (uint32_t)lane;
    bool live = i < np;
    uint32_t o = 0xffffffffu, j = 0;
    V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
    if (live) {
      o = P.key_s[i];
      j = P.val_s[i];
      live = wf_get_ray(S, lv, d, j, y_first, band_rows, band_pitch, n_rows, &ro, &rd);
    }
    const CullRay cr = cull_ray(ro, rd);
    double best = INFINITY;
    uint64_t todo = __ballot(live);
    while (todo) {
      const uint32_t ou = (uint32_t)__builtin_amdgcn_readlane((int)o, (int)__builtin_ctzll(todo));
      const uint64_t mine = __ballot(live && o == ou);
      todo &= ~mine;
      if ((mine >> lane) & 1) best = wfp_object_nearest(D, (int)ou, ro, rd, cr);
    }
    if (live) {
      P.tp[i] = best;
      if (best < INFINITY) atomicMin(&P.tmin[j], (unsigned long long)__double_as_longlong(best));
    }
  }
}

__global__ __launch_bounds__(256) void wfp_near_tie_kernel(WfPairs P) {
  const uint32_t np = min(P.count[0], P.cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < np; i += gridDim.x * blockDim.x) {
    const double t = P.tp[i];
    if (!(t < INFINITY)) continue;
    const uint32_t j = P.val_s[i];
    if ((unsigned long long)__double_as_longlong(t) == P.tmin[j]) atomicMin(&P.omin[j], (int32_t)P.key_s[i]);
  }
}

// Per ray of the level, after the nearest-hit folds: the hit point (wf_ray_core's p) and a coherence
// key for the shadow and shading passes: the hit object above the top `cbits` bits of the Morton code
// of the hit point's cell (a wave then shades one object -- shade_inputs' waterfall runs once -- and
// its shadow rays start close together); misses sort last.
__global__ __launch_bounds__(256) void wfp_hit_key_kernel(RtDevScene S, WfArena A, WfPairs P, int d, uint32_t n,
                                                          int y_first, int band_rows, int band_pitch, int n_rows,
                                                          int cbits) {
  const WfLevel lv = wf_level(A, d);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t j = (d > 0 && A.perm) ? A.perm[i] : i;
    V3 ro, rd;
    uint32_t key = (uint32_t)S.n_objects << cbits;
    if (wf_get_ray(S, lv, d, j, y_first, band_rows, band_pitch, n_rows, &ro, &rd) && P.omin[j] != 0x7fffffff) {
      const V3 p = add(ro, scale(rd, __longlong_as_double((long long)P.tmin[j])));
      P.px[j] = p.x; P.py[j] = p.y; P.pz[j] = p.z;
      const uint32_t cell = (wf_key(A, p, V3{0.0, 0.0, 0.0}) & 0x07ffffffu) >> (27 - cbits);
      key = ((uint32_t)P.omin[j] << cbits) | (cbits ? cell : 0u);
    }
    P.hkey[i] = key;
    P.hval[i] = j;
  }
}

__global__ __launch_bounds__(64) void wfp_shadow_eval_kernel(RtDevScene S, WfPairs P) {
  const int lane = threadIdx.x & 63;
  const uint32_t np = min(P.count[1], P.cap);               // pairs of this level's shadow pass (device)
  const DS D = make_ds(S);
  for (uint32_t base = blockIdx.x * 64u; base < np; base += gridDim.x * 64u) {   // wave-uniform bounds
    const uint32_t i = base + (uint32_t)lane;
    const bool live = i < np;
    uint32_t o = 0xffffffffu, s = 0;
    V3 p = {0.0, 0.0, 0.0}, sdir = {0.0, 0.0, 0.0};
    double ll = 0.0;
    if (live) {
      o = P.key_s[i];
      s = P.val_s[i];
      const uint32_t j = s / (uint32_t)S.n_lights, k = s % (uint32_t)S.n_lights;
      p = {P.px[j], P.py[j], P.pz[j]};
      const RtLight& lt = S.lights[k];
      const V3 l = sub(V3{lt.p[0], lt.p[1], lt.p[2]}, p);              // wf_ray_core's light loop
      double ill;
      len_inv(l, &ll, &ill);
      sdir = scale(l, ill);
    }
    const CullRay cr = cull_ray(p, sdir);
    uint32_t cnt = 0;
    uint64_t todo = __ballot(live);
    while (todo) {
      const uint32_t ou = (uint32_t)__builtin_amdgcn_readlane((int)o, (int)__builtin_ctzll(todo));
      const uint64_t mine = __ballot(live && o == ou);
      todo &= ~mine;
      if ((mine >> lane) & 1) cnt = wfp_object_shadow(D, (int)ou, p, sdir, ll, cr);
    }
    if (live && cnt) {
      if (D.objects[o].transparency == 0.0) atomicOr(&P.opq[s], 1u);
      else atomicAdd(&P.kcnt[s], cnt);
    }
  }
}

template <bool REFR, bool FC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU_WF))) void wfp_shade_kernel(
    RtDevScene S, WfArena A, WfPairs P, int d, uint32_t n, int y_first, int band_rows, int band_pitch, int n_rows,
    int max_depth) {
  const int lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 64u + (uint32_t)lane;
  const WfLevel lv = wf_level(A, d);
  bool live = i < n;
  V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
  uint32_t j = i;
  int32_t pix = (int32_t)i;
  if (live) {
    j = P.hperm[i];                                          // hit-point order (wfp_hit_key_kernel)
    live = wf_get_ray(S, lv, d, j, y_first, band_rows, band_pitch, n_rows, &ro, &rd);
    pix = d > 0 ? lv.pix[j] : (int32_t)j;
  }
  Col L = {0.0, 0.0, 0.0};
  double wt = 0.0, wr = 0.0;
  bool ch_t = false, ch_r = false;
  V3 p = {0.0, 0.0, 0.0}, dt = {0.0, 0.0, 0.0}, dr = {0.0, 0.0, 0.0};
  const uint32_t nl = (uint32_t)S.n_lights;
  const double T = S.shadow_t;
  if (live)
    wf_ray_core<REFR, FC>(
        make_ds(S), ro, rd, d, max_depth,
        [&](double* t) {
          const int32_t oi = P.omin[j];
          if (oi == 0x7fffffff) { *t = INFINITY; return -1; }
          *t = __longlong_as_double((long long)P.tmin[j]);
          return (int)oi;
        },
        [&](int k, V3, V3, double) {
          const uint32_t s = j * nl + (uint32_t)k;
          if (P.opq[s]) return 0.0;
          double tr = 1.0;                                     // shadow_transparency's product, order-free
          for (uint32_t c = P.kcnt[s]; c > 0; --c) {
            tr *= T;
            if (tr == 0.0) return 0.0;
          }
          return tr;
        },
        &L, &wt, &wr, &ch_t, &ch_r, &p, &dt, &dr);
  wf_append(A, lv, d, lane, live, j, pix, L, wt, wr, ch_t, ch_r, p, dt, dr, live ? P.omin[j] : -1);
}

template <bool REFR>
__global__ void record_ray_kernel(RtDevScene S, double x, double y, int max_depth, RtRayRecord* rec, int* order,
                                  int cap, int* counts) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const DS D = make_ds(S);
  BufRec R{rec, order, cap, 0, 0, &D};
  V3 ro, rd;
  camera_ray(S.cam, x, y, &ro, &rd);
  const Col c = trace<REFR, BufRec>(D, ro, rd, max_depth, &R);
  counts[0] = R.n_begun;
  counts[1] = R.n_done;
  rec[cap].color[0] = c.r; rec[cap].color[1] = c.g; rec[cap].color[2] = c.b; rec[cap].color[3] = 1.0;   // get_pixel's return
}

template <bool REFR>
__global__ __launch_bounds__(256) void render_points_kernel(RtDevScene S, const double* __restrict__ xy,
                                                            size_t n, int max_depth, double* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  V3 ro, rd;
  camera_ray(S.cam, xy[2 * i], xy[2 * i + 1], &ro, &rd);
  const Col c = trace<REFR>(make_ds(S), ro, rd, max_depth);
  out[4 * i] = c.r; out[4 * i + 1] = c.g; out[4 * i + 2] = c.b; out[4 * i + 3] = 1.0;
}

// ====================================================================== adaptive anti-aliasing
// antialiaser.rs:87-191 as driven by debug_window.rs:275-320, breadth-first instead of the
// reference's depth-first memoised recursion (same decisions, same traced sub-pixel set, same
// arithmetic):
//   aa_classify  one thread per pixel: the root cell's corners come from the QUANTISED frame
//                (u8 / 255); non-edge pixels are finished here, edge pixels are compacted into a
//                list with one ballot + one atomic per wave;
//   aa_expand    pass p = 1..level, one thread per edge pixel: walk the cell tree to depth p-1,
//                every cell there that subdivides requests its five new grid points (the per-pixel
//                have-mask is the reference's Option<Color> memo);
//   aa_trace     one thread per requested sub-pixel: get_pixel(x + sx/size, y + sy/size);
//   aa_resolve   one thread per edge pixel: the reference recursion over the filled grid.
// Grid points are [sx][sy] as sub_pixels[sub_x][sub_y] (antialiaser.rs:96-99).
struct AaCol { double r, g, b, a; };

__device__ __forceinline__ AaCol aa_src(const uint8_t* src, size_t stride, int x, int y) {   // easy_pixbuf.rs:55-64
  const uint8_t* p = src + (size_t)y * stride + (size_t)x * 4;
  return {p[0] / 255.0, p[1] / 255.0, p[2] / 255.0, p[3] / 255.0};
}
__device__ __forceinline__ bool aa_diff(AaCol c1, AaCol c2, double th) {                   // :154-162
  return (fabs(c1.r - c2.r) + fabs(c1.g - c2.g) + fabs(c1.b - c2.b) + fabs(c1.a - c2.a)) / 4.0 > th;
}
__device__ __forceinline__ AaCol aa_avg(AaCol c1, AaCol c2, AaCol c3, AaCol c4) {           // :164-171
  return {(c1.r + c2.r + c3.r + c4.r) / 4.0, (c1.g + c2.g + c3.g + c4.g) / 4.0,
          (c1.b + c2.b + c3.b + c4.b) / 4.0, (c1.a + c2.a + c3.a + c4.a) / 4.0};
}
__device__ __forceinline__ void aa_put(AaCol c, int x, int y, uint8_t* u8, size_t u8_stride, double* f64,
                                       size_t f64_stride) {
  if (u8) ((uint32_t*)(u8 + (size_t)y * u8_stride))[x] = to_u8(c.r) | (to_u8(c.g) << 8) | (to_u8(c.b) << 16) | (to_u8(c.a) << 24);
  if (f64) {
    double* o = (double*)((uint8_t*)f64 + (size_t)y * f64_stride) + (size_t)x * 4;
    o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = c.a;
  }
}

struct AaGrid {             // per edge pixel: size*size colours + have bits
  AaCol* col;
  uint64_t* have;           // RT_AA_HAVE_WORDS words per edge pixel
  int size;
};
#define RT_AA_MAX_LEVEL 4
#define RT_AA_HAVE_WORDS 5  // (2^4 + 1)^2 = 289 bits

__global__ __launch_bounds__(256) void aa_classify_kernel(const uint8_t* __restrict__ src, size_t stride, int W, int H,
                                                          double th, int level, uint8_t* u8, size_t u8_stride,
                                                          double* f64, size_t f64_stride, uint32_t* __restrict__ edges,
                                                          uint32_t* __restrict__ n_edges) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_x = (W + 15) >> 4;
  const int x = ((blockIdx.x % tiles_x) << 4) + ((wave & 1) << 3) + (lane & 7);
  const int y = ((blockIdx.x / tiles_x) << 4) + ((wave >> 1) << 3) + (lane >> 3);
  bool edge = false;
  if (x < W && y < H) {
    if (x == W - 1 || y == H - 1) {          // last column copied (:67-68); last row never touched (debug_window.rs:298)
      aa_put(aa_src(src, stride, x, y), x, y, u8, u8_stride, f64, f64_stride);
    } else {
      const AaCol c1 = aa_src(src, stride, x, y), c2 = aa_src(src, stride, x + 1, y);
      const AaCol c3 = aa_src(src, stride, x, y + 1), c4 = aa_src(src, stride, x + 1, y + 1);
      edge = level > 0 && (aa_diff(c1, c2, th) || aa_diff(c1, c3, th) || aa_diff(c1, c4, th));
      if (!edge) aa_put(aa_avg(c1, c2, c3, c4), x, y, u8, u8_stride, f64, f64_stride);
    }
  }
  const uint64_t m = __ballot(edge);                                   // wave-aggregated compaction
  if (m == 0) return;
  uint32_t base = 0;
  if (lane == __ffsll((long long)m) - 1) base = atomicAdd(n_edges, (uint32_t)__popcll(m));
  base = __shfl(base, __ffsll((long long)m) - 1);
  if (edge) edges[base + __popcll(m & ((1ull << lane) - 1))] = ((uint32_t)y << 16) | (uint32_t)x;
}

__device__ __forceinline__ bool aa_has(const uint64_t* h, int i) { return (h[i >> 6] >> (i & 63)) & 1u; }

// Depth-first walk to depth `target`; cells there that subdivide request their new points
// (have = the pixel's memo bits, updated).  With req == nullptr only counts; otherwise writes the
// requests to req[base ...].  Returns the number of new points.
__device__ uint32_t aa_expand_cell(const AaGrid& G, uint32_t e, int target, int level, double th, uint64_t* have,
                                   uint2* req, uint32_t base) {
  struct Frame { int8_t x1, y1, x2, y2, depth; };
  Frame st[4 * RT_AA_MAX_LEVEL + 4];
  int sp = 0;
  const int sz = G.size;
  st[sp++] = {0, 0, (int8_t)(sz - 1), (int8_t)(sz - 1), 0};
  const AaCol* col = G.col + (size_t)e * sz * sz;
  uint32_t n = 0;
  while (sp > 0) {
    const Frame f = st[--sp];
    const AaCol c1 = col[f.x1 * sz + f.y1], c2 = col[f.x2 * sz + f.y1];
    const AaCol c3 = col[f.x1 * sz + f.y2], c4 = col[f.x2 * sz + f.y2];
    const bool split = (level - f.depth) > 0 && (aa_diff(c1, c2, th) || aa_diff(c1, c3, th) || aa_diff(c1, c4, th));
    if (!split) continue;
    const int mx = f.x1 + (f.x2 - f.x1) / 2, my = f.y1 + (f.y2 - f.y1) / 2;
    if (f.depth < target) {                                    // children, pushed so the first pops first
      st[sp++] = {(int8_t)mx, (int8_t)my, f.x2, f.y2, (int8_t)(f.depth + 1)};
      st[sp++] = {f.x1, (int8_t)my, (int8_t)mx, f.y2, (int8_t)(f.depth + 1)};
      st[sp++] = {(int8_t)mx, f.y1, f.x2, (int8_t)my, (int8_t)(f.depth + 1)};
      st[sp++] = {f.x1, f.y1, (int8_t)mx, (int8_t)my, (int8_t)(f.depth + 1)};
      continue;
    }
    const int px[5] = {mx, f.x1, mx, f.x2, mx}, py[5] = {f.y1, my, my, my, f.y2};
    for (int k = 0; k < 5; ++k) {
      const int i = px[k] * sz + py[k];
      if (aa_has(have, i)) continue;
      have[i >> 6] |= 1ull << (i & 63);
      if (req) req[base + n] = make_uint2(e, (uint32_t)(px[k] | (py[k] << 8)));
      ++n;
    }
  }
  return n;
}

__global__ __launch_bounds__(256) void aa_init_kernel(AaGrid G, const uint8_t* __restrict__ src, size_t stride,
                                                      const uint32_t* __restrict__ edges, uint32_t n) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int x = edges[e] & 0xffff, y = edges[e] >> 16, sz = G.size, nn = sz - 1;
  AaCol* col = G.col + (size_t)e * sz * sz;
  uint64_t* h = G.have + (size_t)e * RT_AA_HAVE_WORDS;
  for (int w = 0; w < RT_AA_HAVE_WORDS; ++w) h[w] = 0;
  const int idx[4] = {0, nn, nn * sz, nn * sz + nn};                  // [0][0] [0][n] [n][0] [n][n] (:96-99)
  col[idx[0]] = aa_src(src, stride, x, y);
  col[idx[1]] = aa_src(src, stride, x, y + 1);
  col[idx[2]] = aa_src(src, stride, x + 1, y);
  col[idx[3]] = aa_src(src, stride, x + 1, y + 1);
  for (int k = 0; k < 4; ++k) h[idx[k] >> 6] |= 1ull << (idx[k] & 63);
}

__global__ __launch_bounds__(256) void aa_expand_kernel(AaGrid G, uint32_t n, int pass, int level, double th,
                                                        uint2* __restrict__ req, uint32_t* __restrict__ n_req,
                                                        uint32_t cap) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = e < n;
  uint64_t have[RT_AA_HAVE_WORDS], probe[RT_AA_HAVE_WORDS];
  uint32_t cnt = 0;
  if (live) {
    const uint64_t* h = G.have + (size_t)e * RT_AA_HAVE_WORDS;
    for (int w = 0; w < RT_AA_HAVE_WORDS; ++w) probe[w] = have[w] = h[w];
    cnt = aa_expand_cell(G, e, pass - 1, level, th, probe, nullptr, 0);   // count
  }
  // one atomic per wave: exclusive prefix of the lane counts
  const int lane = threadIdx.x & 63;
  uint32_t incl = cnt;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d);
    if (lane >= d) incl += v;
  }
  const uint32_t total = __shfl(incl, 63);
  uint32_t base = 0;
  if (lane == 63 && total > 0) base = atomicAdd(n_req, total);
  base = __shfl(base, 63) + (incl - cnt);
  if (!live || cnt == 0) return;
  if (base + cnt > cap) return;                                          // host reports the overflow
  aa_expand_cell(G, e, pass - 1, level, th, have, req, base);            // write
  uint64_t* h = G.have + (size_t)e * RT_AA_HAVE_WORDS;
  for (int w = 0; w < RT_AA_HAVE_WORDS; ++w) h[w] = have[w];
}

// One-wave workgroups with the frame stack's first frames in LDS, as the row kernels.
template <bool REFR, bool FC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES(REFR)))) void aa_trace_kernel(
    RtDevScene S, AaGrid G, const uint32_t* __restrict__ edges, const uint2* __restrict__ req, uint32_t n, int max_depth) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  constexpr int KLR = REFR ? RT_LDS_RFRAMES : 0;
  __shared__ double s_frames[(RT_LDS_FRAMES * 4 + KLR * 7) * 64 + 1];
  lds_f64* lf = (lds_f64*)&s_frames[threadIdx.x];
  if (i >= n) return;
  const uint2 r = req[i];
  const int x = edges[r.x] & 0xffff, y = edges[r.x] >> 16;
  const int sx = r.y & 0xff, sy = r.y >> 8, sz = G.size;
  V3 ro, rd;
  camera_ray(S.cam, (double)x + ((double)sx / (double)sz), (double)y + ((double)sy / (double)sz), &ro, &rd);   // :108-112
  const Col c = trace<REFR, NoRec, RT_LDS_FRAMES, FC, KLR>(make_ds(S), ro, rd, max_depth, nullptr, lf);
  G.col[(size_t)r.x * sz * sz + sx * sz + sy] = {c.r, c.g, c.b, 1.0};
}

// get_sub_pixel_color (:124-152) over the filled grid; D bounds the remaining depth at compile time.
// Fully inlined (256 VGPRs, no scratch): measured faster than an explicit-stack loop, whose frame
// array lives in scratch (profiles/r01j_aa_timing.txt).
template <int D>
__device__ AaCol aa_cell(const AaCol* col, int sz, int x1, int y1, int x2, int y2, int lv, double th) {
  const AaCol c1 = col[x1 * sz + y1], c2 = col[x2 * sz + y1], c3 = col[x1 * sz + y2], c4 = col[x2 * sz + y2];
  if constexpr (D == 0) {
    return aa_avg(c1, c2, c3, c4);
  } else {
    if (!(aa_diff(c1, c2, th) || aa_diff(c1, c3, th) || aa_diff(c1, c4, th)) || lv <= 0) return aa_avg(c1, c2, c3, c4);
    const int mx = x1 + (x2 - x1) / 2, my = y1 + (y2 - y1) / 2;
    const AaCol k1 = aa_cell<D - 1>(col, sz, x1, y1, mx, my, lv - 1, th);
    const AaCol k2 = aa_cell<D - 1>(col, sz, mx, y1, x2, my, lv - 1, th);
    const AaCol k3 = aa_cell<D - 1>(col, sz, x1, my, mx, y2, lv - 1, th);
    const AaCol k4 = aa_cell<D - 1>(col, sz, mx, my, x2, y2, lv - 1, th);
    return aa_avg(k1, k2, k3, k4);
  }
}

__global__ __launch_bounds__(256) void aa_resolve_kernel(AaGrid G, const uint32_t* __restrict__ edges, uint32_t n,
                                                         int level, double th, uint8_t* u8, size_t u8_stride,
                                                         double* f64, size_t f64_stride) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int sz = G.size;
  const AaCol* col = G.col + (size_t)e * sz * sz;
  const AaCol res = aa_cell<RT_AA_MAX_LEVEL>(col, sz, 0, 0, sz - 1, sz - 1, level, th);
  aa_put(res, edges[e] & 0xffff, edges[e] >> 16, u8, u8_stride, f64, f64_stride);
}

// ====================================================================== orthogonal preview views
// DebugWindow::render_orthogonal_view_line (debug_window.rs:166-227): a ray from 10000 along the
// view axis per pixel; the object with the smallest intersection distance -- ANY sign, no EPS,
// strict `<` so the first emitted wins ties -- gives its flat colour (RTObject::get_color =
// material colour at uv (0,0), rt_object.rs:45-47); a miss is Color::EMPTY.  No culling: t may
// be negative.
struct OrthoView { int axis1, axis2, axis3; double dir1, dir2, scale; };

__global__ __launch_bounds__(256) void ortho_kernel(RtDevScene S, OrthoView V, int y0, int n_rows,
                                                    uint8_t* __restrict__ out, size_t stride,
                                                    double* __restrict__ f64, size_t f64_stride) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_x = (S.width + 15) >> 4;
  const int x = ((blockIdx.x % tiles_x) << 4) + ((wave & 1) << 3) + (lane & 7);
  const int r = ((blockIdx.x / tiles_x) << 4) + ((wave >> 1) << 3) + (lane >> 3);
  if (x >= S.width || r >= n_rows) return;
  const int y = y0 + r;
  const DS D = make_ds(S);
  const double cx = (double)S.width / 2.0, cy = (double)S.height / 2.0;
  double o3[3] = {0.0, 0.0, 0.0}, d3[3] = {0.0, 0.0, 0.0};
  o3[V.axis1] = (((double)x - cx) * V.dir1) / V.scale;
  o3[V.axis2] = (((double)y - cy) * V.dir2) / V.scale;
  o3[V.axis3] = 10000.0;
  d3[V.axis3] = 1.0;
  const V3 ro = {o3[0], o3[1], o3[2]}, rd = {d3[0], d3[1], d3[2]};
  double best = INFINITY;
  int bobj = -1;
  const bool fin = wave_finite(ro, rd);
  for (int o = 0; o < D.n_objects; ++o) {
    cptr<RtObject> O = &D.objects[o];
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    for (int l = lb; l < le; ++l) {
      cptr<RtLeaf> L = &D.leaves[l];
      double t0 = 0.0, t1 = 0.0;
      const int n = leaf_candidates(L, ro, rd, fin, &t0, &t1);
      const bool filtered = L->prog_end != L->prog_begin;
      if (n >= 1 && t0 < best && (!filtered || leaf_filter(D, L, add(ro, scale(rd, t0))))) { best = t0; bobj = o; }
      if (n >= 2 && t1 < best && (!filtered || leaf_filter(D, L, add(ro, scale(rd, t1))))) { best = t1; bobj = o; }
    }
  }
  double c[4] = {0.0, 0.0, 0.0, 0.0};                                     // Color::EMPTY
  if (bobj >= 0) {
    cptr<RtObject> O = &D.objects[bobj];
    if (O->textured) {                                                     // texture.rs:27-34 at (0, 0)
      const int tw = D.textures[O->tex].w, th = D.textures[O->tex].h;
      const double ty = (double)th - (0.0 * (double)(th - 1)) - 1.0;
      const int yi = ty > 0.0 ? (ty < (double)(th - 1) ? (int)ty : th - 1) : 0;
      const uint32_t px = *(const uint32_t*)(D.texels + D.textures[O->tex].offset + (size_t)yi * tw * 4);
      c[0] = (double)(px & 0xffu) / 255.0; c[1] = (double)((px >> 8) & 0xffu) / 255.0;
      c[2] = (double)((px >> 16) & 0xffu) / 255.0; c[3] = (double)(px >> 24) / 255.0;
    } else {
      c[0] = O->color[0]; c[1] = O->color[1]; c[2] = O->color[2]; c[3] = O->color_a;
    }
  }
  if (out) ((uint32_t*)(out + (size_t)r * stride))[x] = to_u8(c[0]) | (to_u8(c[1]) << 8) | (to_u8(c[2]) << 16) | (to_u8(c[3]) << 24);
  if (f64) {
    double* p = (double*)((uint8_t*)f64 + (size_t)r * f64_stride) + (size_t)x * 4;
    p[0] = c[0]; p[1] = c[1]; p[2] = c[2]; p[3] = c[3];
  }
}

// ====================================================================== multi-GPU frame assembly
// Row-band layout (distributed.py): frame row y is in band b = y / band_rows, dealt to rank
// b % world, which packed it at slot row (b / world) * band_rows + y % band_rows.  After the
// all-gather (slots in rank order) one launch puts every row at its y -- the GTK thread's
// apply_line (debug_window.rs:147-163) for all ranks at once.  A contiguous tile per rank is the
// case band_rows = slot_rows.  One workgroup per row, 16-byte copies when every address allows.
__global__ __launch_bounds__(256) void assemble_bands_kernel(const uint8_t* __restrict__ g, size_t gstride, int world,
                                                             int slot_rows, int band, size_t row_bytes,
                                                             uint8_t* __restrict__ f, size_t fstride, int vec16) {
  const int y = blockIdx.x, b = y / band;
  const uint8_t* s = g + ((size_t)(b % world) * slot_rows + (size_t)(b / world) * band + y % band) * gstride;
  uint8_t* d = f + (size_t)y * fstride;
  if (vec16) {
    for (size_t i = threadIdx.x; i < row_bytes / 16; i += blockDim.x) ((uint4*)d)[i] = ((const uint4*)s)[i];
  } else {
    for (size_t i = threadIdx.x; i < row_bytes; i += blockDim.x) d[i] = s[i];
  }
}

// The same placement from packed RGB8 slot rows (3 bytes per pixel, rt_render_row_bands_rgb8) into
// RGBA8 frame rows with A = 255: the all-gather moves 3/4 of the bytes.  One workgroup per row.
// vec: 4 pixels per thread and iteration -- three 4-byte loads (12 bytes = 4 RGB pixels) and one
// 16-byte store -- when the slot rows are 4-byte and the frame rows 16-byte aligned and the width
// is a multiple of 4; otherwise one pixel per thread (3 byte loads, one 4-byte store).
__global__ __launch_bounds__(256) void assemble_bands_rgb_kernel(const uint8_t* __restrict__ g, size_t gstride,
                                                                 int world, int slot_rows, int band, int width,
                                                                 uint8_t* __restrict__ f, size_t fstride, int vec) {
  const int y = blockIdx.x, b = y / band;
  const uint8_t* s = g + ((size_t)(b % world) * slot_rows + (size_t)(b / world) * band + y % band) * gstride;
  uint32_t* d = (uint32_t*)(f + (size_t)y * fstride);
  if (vec) {
    const uint32_t* s4 = (const uint32_t*)s;
    for (int q = threadIdx.x; q < width / 4; q += blockDim.x) {
      const uint32_t w0 = s4[3 * q], w1 = s4[3 * q + 1], w2 = s4[3 * q + 2];
      uint4 o;
      o.x = (w0 & 0xFFFFFFu) | 0xFF000000u;
      o.y = (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | 0xFF000000u;
      o.z = (w1 >> 16) | ((w2 & 0xFFu) << 16) | 0xFF000000u;
      o.w = (w2 >> 8) | 0xFF000000u;
      ((uint4*)d)[q] = o;
    }
    return;
  }
  for (int x = threadIdx.x; x < width; x += blockDim.x) {
    const uint8_t* p = s + (size_t)x * 3;
    d[x] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | (255u << 24);
  }
}

}  // namespace

// ====================================================================== device context
struct rt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;       // last stream launched on (NULL = the default stream)
  void* d_blob = nullptr;
  size_t blob_bytes = 0;
  RtDevScene dev;
  int32_t max_depth = 10;
  int32_t kernel_opt = RT_KERNEL_AUTO;  // rt_ctx_set_option(RT_OPT_KERNEL)
  bool timing = true;                   // rt_ctx_set_option(RT_OPT_TIMING): launch events recorded
  bool tile_order = true;               // rt_ctx_set_option(RT_OPT_TILE_ORDER): cost-ordered dispatch
  bool fast_clamp = true;               // rt_ctx_set_option(RT_OPT_FAST_CLAMP): min/max clamps where exact
  int wf_cap_pct = 200;                 // rt_ctx_set_option(RT_OPT_WAVEFRONT_CAP): rays per level, % of pixel slots
  double wf_klo[3] = {-100, -100, -100}, wf_khi[3] = {100, 100, 100};   // coherence-key extent (bounded objects)
  int n_cu = 256;                       // compute units of the device (wave slots = n_cu x 4 SIMDs x waves/SIMD)
  bool uploaded = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t tev0 = nullptr, tev1 = nullptr;   // the wavefront autotune's own pair
  bool timed = false;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* wf = nullptr;                   // wavefront arena (levels, counters, overflow flags), grow-only
  size_t wf_bytes = 0;
  int wf_pairs = 1;                     // rt_ctx_set_option(RT_OPT_WAVEFRONT_PAIRS): 0 off, 1 levels >= 1, 2 every level
  void* wfr = nullptr;                  // pair path: per-ray arrays (nearest hit, hit point, shadow counts), grow-only
  size_t wfr_bytes = 0;
  void* wfp = nullptr;                  // pair path: pair lists + sort scratch, grow-only
  size_t wfp_bytes = 0;
  uint32_t wfp_cap = 0;
  // Cost-ordered tile dispatch.  A frame's time is set by its slowest tiles (long reflection
  // chains), so they are dispatched first: the first launch of a geometry records every tile's
  // wave time, and later launches of the same geometry read the tiles in descending cost order.
  // One table per geometry key (rows, bands, depth, f64, width), RT_ORDER_SLOTS of them, LRU.
  // A table is written exactly once (its calibration, synchronous) and never rewritten while it
  // exists, so launches queued on other streams can never read a half-written order; tables are
  // freed only by hipFree (which waits for the device) on eviction, upload or rt_ctx_free.
  struct OrderSlot {
    int32_t key[7] = {0};
    int32_t* d_order = nullptr;
    uint32_t* d_cost = nullptr;
    size_t n_tiles = 0;
    uint32_t grid = 0;                // entries of the order (> n_tiles when costly tiles are split)
    uint64_t last_use = 0;
    bool deferred = false;            // ordered launches take the deferred-shadow kernel
    int wf_tune = 0;                  // ray-tree scenes, RT_KERNEL_AUTO: 0 not yet timed, 1 megakernel, 2 wavefront
    bool valid = false;               // set once the sorted order is on the device
  };
  static constexpr int RT_ORDER_SLOTS = 8;
  OrderSlot order[RT_ORDER_SLOTS];
  uint64_t use_clock = 0;
};

using rt::fail;

#define RT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

// Environment: RT_TILE_ORDER_DEBUG=1 prints each calibration's tile-cost statistics and the kernel
// it picked to stderr (diagnostic).  Every tunable is a context option (rt_ctx_set_option).

// Kernel choice for scenes without a transparent object (REFR = false), RT_OPT_KERNEL AUTO:
//   * launches of fewer than RT_ORDER_MIN_TILES tiles (no calibration) take the deferred kernel;
//   * larger launches calibrate on the megakernel; the ordered launches that follow take the
//     deferred kernel with split tiles when the launch has fewer than RT_DEFERRED_MAX_TILES tiles
//     AND its costliest tile is longer than the work per wave slot (sum of tile costs / the chip's
//     wave slots for the calibrated kernel: CUs x 4 SIMDs x its waves per SIMD): then the tail,
//     not the throughput, sets the time.
// Same pixels either way.  Measured (profiles/r02h_inflight.txt, r02j_*): a rank's share of the
// 4K globes frame at N = 8 / 4 (16320 / 32640 tiles, tail ratio 3.5 / 1.8) takes 0.146-0.178 /
// 0.187-0.204 ms deferred + split against 0.244 / 0.254 ms in the megakernel, 1080p globes d5
// (ratio 1.7) 0.219 against 0.26-0.28 ms; at N = 2 / 1 (64800 / 129600 tiles, ratio 1.0 / 0.5),
// and for the 1080p single sphere (32400 tiles, ratio 0.75: no tail to speak of), the megakernel
// is 7-20 % faster.  The deferred kernel's order entries hold the tile index in 20 bits
// (RT_SPLIT_TILE_MASK), so launches of more tiles always take the megakernel.
#define RT_DEFERRED_MAX_TILES 40000

static void drop_order(rt_ctx::OrderSlot& s) {
  if (s.d_order) (void)hipFree(s.d_order);     // hipFree waits for work that may still read it
  if (s.d_cost) (void)hipFree(s.d_cost);
  s = rt_ctx::OrderSlot();
}
static void drop_orders(rt_ctx* c) {
  for (auto& s : c->order) drop_order(s);
}

// Launches with fewer tiles than this are dispatched row-major without a calibration launch: a
// small band (a single row, one rank's sliver) has no tail worth reordering, and calibrating it
// would cost a host synchronisation per new geometry.
#ifndef RT_ORDER_MIN_TILES
#define RT_ORDER_MIN_TILES 2048
#endif

static int ensure_scratch(rt_ctx* c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return RT_OK;
  if (c->scratch) (void)hipFree(c->scratch);
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  RT_HIP(hipMalloc(&c->scratch, bytes));
  c->scratch_bytes = bytes;
  return RT_OK;
}

static bool is_device_ptr(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

template <typename T>
static size_t put(std::vector<uint8_t>& blob, const std::vector<T>& v) {
  size_t off = (blob.size() + 255) & ~(size_t)255;
  blob.resize(off + v.size() * sizeof(T) + 16);
  if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
  return off;
}

extern "C" {

#ifdef RT_COUNT
__attribute__((visibility("default"))) int rt_diag_cnt(unsigned long long* out64) {
  if (hipDeviceSynchronize() != hipSuccess) return RT_ERR_DEVICE;
  if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_rt_cnt), 64 * sizeof(unsigned long long)) != hipSuccess) return RT_ERR_DEVICE;
  static const unsigned long long zero[64] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_rt_cnt), zero, sizeof(zero)) != hipSuccess) return RT_ERR_DEVICE;
  return RT_OK;
}
#endif

#ifdef RT_DIAG_ENTRY_TIMES
// Diagnostic build only: start / end wall-clock ticks (100 MHz) of each entry of the last ordered
// deferred launch, and the order itself (entry -> tile | part << 20 | log2 P << 24).
__attribute__((visibility("default"))) int rt_diag_entry_times(rt_ctx* c, uint64_t* out, int32_t* order, size_t n) {
  if (hipDeviceSynchronize() != hipSuccess) return RT_ERR_DEVICE;
  if (n > RT_ENTRY_TIMES_MAX) n = RT_ENTRY_TIMES_MAX;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_entry_times), n * 16) != hipSuccess) return RT_ERR_DEVICE;
  for (auto& s : c->order)
    if (s.valid && s.deferred)
      return hipMemcpy(order, s.d_order, std::min<size_t>(n, s.grid) * 4, hipMemcpyDeviceToHost) == hipSuccess ? 0 : RT_ERR_DEVICE;
  return RT_ERR_INVALID;
}
#endif
#ifdef RT_TILE_STATS
// Diagnostic build only: the per-tile stats of the last calibration launch (4 words per tile).
__attribute__((visibility("default"))) int rt_diag_tile_stats(uint32_t* out, size_t n_tiles) {
  if (hipDeviceSynchronize() != hipSuccess) return RT_ERR_DEVICE;
  if (n_tiles > RT_STATS_TILES) n_tiles = RT_STATS_TILES;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tile_stats), n_tiles * 16) != hipSuccess) return RT_ERR_DEVICE;
  return RT_OK;
}
#endif

#ifdef RT_PROF
// Diagnostic build only: read-and-reset the section wave-cycle counters (tools/section_profile.py).
__attribute__((visibility("default"))) int rt_diag_prof(unsigned long long* out8) {
  if (hipDeviceSynchronize() != hipSuccess) return RT_ERR_DEVICE;
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_rt_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return RT_ERR_DEVICE;
  static const unsigned long long zero[8] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_rt_prof), zero, sizeof(zero)) != hipSuccess) return RT_ERR_DEVICE;
  return RT_OK;
}
#endif

int rt_device_count(int* count) {
  if (!count) return fail(RT_ERR_INVALID, "null output");
  *count = 0;
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) { *count = 0; return fail(RT_ERR_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e)); }
  return RT_OK;
}

int rt_ctx_create(int device, rt_ctx** out) {
  if (!out) return fail(RT_ERR_INVALID, "null output");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RT_ERR_DEVICE, "no HIP device available");
  if (device < 0 || device >= n) return fail(RT_ERR_INVALID, "device %d out of range (%d devices)", device, n);
  RT_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  RT_HIP(hipGetDeviceProperties(&prop, device));
  rt_ctx* c = new rt_ctx();
  c->device = device;
  c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  memset(&c->dev, 0, sizeof c->dev);
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->tev0) != hipSuccess || hipEventCreate(&c->tev1) != hipSuccess) {
    delete c;
    return fail(RT_ERR_DEVICE, "stream/event creation failed");
  }
  *out = c;
  return RT_OK;
}

int rt_ctx_upload(rt_ctx* c, const rt_scene* s) {
  if (!c || !s) return fail(RT_ERR_INVALID, "null argument");
  rt::FlatScene f;
  int rc = rt::flatten(*s, &f);
  if (rc) return rc;
  std::vector<uint8_t> blob;
  size_t o_obj = put(blob, f.objects), o_trav = put(blob, f.trav), o_strav = put(blob, f.strav), o_nodes = put(blob, f.nodes),
         o_leaves = put(blob, f.leaves);
  size_t o_prog = put(blob, f.prog), o_lights = put(blob, f.lights), o_tex = put(blob, f.textures);
  size_t o_texels = put(blob, f.texels);
  RT_HIP(hipSetDevice(c->device));
  if (c->d_blob) { (void)hipFree(c->d_blob); c->d_blob = nullptr; }
  c->uploaded = false;
  RT_HIP(hipMalloc(&c->d_blob, blob.size()));
  RT_HIP(hipMemcpy(c->d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
  c->blob_bytes = blob.size();
  uint8_t* b = (uint8_t*)c->d_blob;
  RtDevScene& d = c->dev;
  d.objects = (const RtObject*)(b + o_obj);
  d.trav = (const RtTrav*)(b + o_trav);
  d.n_trav = (int32_t)f.trav.size();
  d.strav = (const RtTrav*)(b + o_strav);
  d.n_strav = (int32_t)f.strav.size();
  d.nodes = (const RtNode*)(b + o_nodes);
  d.leaves = (const RtLeaf*)(b + o_leaves);
  d.prog = (const RtProg*)(b + o_prog);
  d.lights = (const RtLight*)(b + o_lights);
  d.textures = (const RtTexture*)(b + o_tex);
  d.texels = b + o_texels;
  d.n_objects = (int32_t)f.objects.size();
  d.n_lights = (int32_t)f.lights.size();
  d.n_leaves = (int32_t)f.leaves.size();
  d.n_nodes = (int32_t)f.nodes.size();
  d.width = f.width;
  d.height = f.height;
  d.any_transparent = f.any_transparent;
  d.shadow_early_out = f.shadow_early_out;
  d.colour_fast = f.colour_fast;
  d.ray_chains = f.ray_chains;
  d.shadow_pow = f.shadow_pow;
  d.shadow_t = f.shadow_t;
  d.cam = f.cam;
  c->max_depth = f.max_depth;
  {                                   // the wavefront path's key extent: the hull of the bounded objects
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const RtObject& o : f.objects)
      if (o.cull == RT_CULL_BOX)
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], o.blo[k]); hi[k] = std::max(hi[k], o.bhi[k]); }
    for (int k = 0; k < 3; ++k) {
      const bool ok = std::isfinite(lo[k]) && std::isfinite(hi[k]) && hi[k] > lo[k];
      c->wf_klo[k] = ok ? lo[k] : f.cam.center[k] - 100.0;
      c->wf_khi[k] = ok ? hi[k] : f.cam.center[k] + 100.0;
    }
  }
  c->uploaded = true;
  drop_orders(c);                     // tile costs belong to the previous scene
  return RT_OK;
}

extern "C" hipError_t rt_wf_bucket_sort(const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                                        uint32_t* vals_out, uint32_t n, const uint32_t* n_dev, uint32_t nb, int shift,
                                        uint32_t* cnt, bool zero_cnt, hipStream_t stream);
extern "C" hipError_t rt_wf_sort_pairs(void* d_temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                       const uint32_t* vals_in, uint32_t* vals_out, int n, int end_bit,
                                       hipStream_t stream);

// Pair-path arrays (render_kernels.hip "wavefront pair path"): per ray of a level (R = the larger of
// the pixel slots and the level capacity) and, grow-only, the pair lists for `need` pairs.
static int wfp_arena(rt_ctx* c, hipStream_t st, size_t R, size_t lcap, size_t need, WfPairs* P) {
  const size_t nl = (size_t)std::max(1, c->dev.n_lights);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_omin = al(R * 8), o_px = al(o_omin + R * 4), o_k = al(o_px + 3 * R * 8), o_q = al(o_k + R * nl * 4);
  const size_t o_h = al(o_q + R * nl * 4), rbytes = al(o_h + 4 * R * 4);
  if (c->wfr_bytes < rbytes) {
    if (c->wfr) (void)hipFree(c->wfr);
    c->wfr = nullptr;
    c->wfr_bytes = 0;
    RT_HIP(hipMalloc(&c->wfr, rbytes));
    c->wfr_bytes = rbytes;
  }
  if (need > c->wfp_cap || !c->wfp) {
    // first size: 4 pairs per ray of a full level (fractal.scene needs ~3); a level that emits more
    // grows it (RT_OPT_WAVEFRONT_CAP 1 % makes the first size tiny: the overflow tests take that path)
    const size_t cap = std::min<size_t>(0x7fffffc0ull, std::max<size_t>(need + need / 4, 4 * lcap) + 63) & ~(size_t)63;
    if (need > cap) return fail(RT_ERR_UNSUPPORTED, "wavefront pair list of %zu pairs too large", need);
    const size_t bytes = al(3 * 16384 + 4 * cap * 4 + cap * 8);
    if (c->wfp) (void)hipFree(c->wfp);    // waits for launches that may still use it
    c->wfp = nullptr;
    c->wfp_bytes = 0;
    c->wfp_cap = 0;
    RT_HIP(hipMalloc(&c->wfp, bytes));
    c->wfp_bytes = bytes;
    c->wfp_cap = (uint32_t)cap;
  }
  uint8_t* r = (uint8_t*)c->wfr;
  P->tmin = (unsigned long long*)r;
  P->omin = (int32_t*)(r + o_omin);
  P->px = (double*)(r + o_px);
  P->py = P->px + R;
  P->pz = P->py + R;
  P->kcnt = (uint32_t*)(r + o_k);
  P->opq = (uint32_t*)(r + o_q);
  P->hkey = (uint32_t*)(r + o_h);
  P->hval = P->hkey + R;
  P->hkey_s = P->hval + R;
  P->hperm = P->hkey_s + R;
  uint8_t* b = (uint8_t*)c->wfp;
  const size_t cap = c->wfp_cap;
  P->cap = (uint32_t)cap;
  P->count = nullptr;                   // set by the caller: the wavefront arena's counter block
  P->bins = (uint32_t*)b;               // 3 x RT_BS_MAX_BINS words: nearest / hit-point / shadow sorts
  P->key = (uint32_t*)(b + 3 * 16384);
  P->val = P->key + cap;
  P->key_s = P->val + cap;
  P->val_s = P->key_s + cap;
  P->tp = (double*)(P->val_s + cap);
  return RT_OK;
}

// One level of the wavefront path through the pair path: candidate pairs, sort by object, pair
// evaluation and the folds, for the nearest hits and then the shadow rays, then the shading pass.
// The pair counts stay on the device (the sorts and the evaluation kernels read them; their grids
// are sized for the arena), so a level costs ONE host synchronisation, at its end: it reads the next
// level's ray count and both pair counts.  A pair count beyond the arena grows it and runs the level
// again (the level's outputs are recomputed from its rays; level d + 1 is refilled from empty).
static int wfp_level(rt_ctx* c, hipStream_t st, const WfArena& A, size_t R, int d, uint32_t n, int a0, int a1,
                     int a2, int a3, int max_depth, bool refr, bool fc, uint32_t* next) {
  WfPairs P;
  int rc = wfp_arena(c, st, R, A.cap, 0, &P);
  if (rc) return rc;
  P.count = A.count + RT_WFP_COUNT;
  const dim3 g((n + 63) / 64), b64(64);
  const uint32_t nobj = (uint32_t)c->dev.n_objects;
  uint32_t* bins[3] = {P.bins, P.bins + 4096, P.bins + 8192};
  for (;;) {
    // grid-stride evaluations: one pass covers ~4 pairs per ray of the level (fractal: ~3), capped at
    // 8 waves per SIMD -- small levels then launch hundreds, not thousands, of idle workgroups
    const dim3 ge(std::max<uint32_t>((uint32_t)c->n_cu, std::min<uint32_t>((uint32_t)(((size_t)n * 4 + 63) / 64),
                                                                          (uint32_t)c->n_cu * 32u)));
    RT_HIP(hipMemsetAsync(P.count, 0, 8, st));
    RT_HIP(hipMemsetAsync(P.bins, 0, 3 * 16384, st));        // the three sorts' bucket counters
    hipLaunchKernelGGL((wfp_cand_kernel<false>), g, b64, 0, st, c->dev, A, P, d, n, a0, a1, a2, a3);
    RT_HIP(rt_wf_bucket_sort(P.key, P.key_s, P.val, P.val_s, P.cap, P.count, nobj, 0, bins[0], false, st));
    hipLaunchKernelGGL(wfp_near_eval_kernel, ge, b64, 0, st, c->dev, A, P, d, a0, a1, a2, a3);
#ifdef RT_DIAG_TWICE                      // diagnostic build only: the (idempotent) evaluation again, warm
    hipLaunchKernelGGL(wfp_near_eval_kernel, ge, b64, 0, st, c->dev, A, P, d, a0, a1, a2, a3);
#endif
    hipLaunchKernelGGL(wfp_near_tie_kernel, dim3(std::min<uint32_t>((P.cap + 255) / 256, 4096)), dim3(256), 0, st, P);
    // the hit points and their order for the shadow and shading passes: at most 4096 buckets of
    // (hit object, coarse hit-point cell), unordered within a bucket (a 16^3-cell-only key and the
    // full 27-bit radix sort measured slower: profiles/r03o_sort_ab.txt, r03w_*)
    int cbits = 0;
    while (cbits < 12 && ((nobj + 1u) << (cbits + 1)) <= 4096u) ++cbits;
    hipLaunchKernelGGL(wfp_hit_key_kernel, dim3(std::min<uint32_t>((n + 255) / 256, 8192)), dim3(256), 0, st, c->dev,
                       A, P, d, n, a0, a1, a2, a3, cbits);
    RT_HIP(rt_wf_bucket_sort(P.hkey, P.hkey_s, P.hval, P.hperm, n, nullptr, (nobj + 1u) << cbits, 0, bins[1], false, st));
    hipLaunchKernelGGL((wfp_cand_kernel<true>), g, b64, 0, st, c->dev, A, P, d, n, a0, a1, a2, a3);
    RT_HIP(rt_wf_bucket_sort(P.key, P.key_s, P.val, P.val_s, P.cap, P.count + 1, nobj, 0, bins[2], false, st));
    hipLaunchKernelGGL(wfp_shadow_eval_kernel, ge, b64, 0, st, c->dev, P);
    if (refr && fc) hipLaunchKernelGGL((wfp_shade_kernel<true, true>), g, b64, 0, st, c->dev, A, P, d, n, a0, a1, a2, a3, max_depth);
    else if (refr) hipLaunchKernelGGL((wfp_shade_kernel<true, false>), g, b64, 0, st, c->dev, A, P, d, n, a0, a1, a2, a3, max_depth);
    else if (fc) hipLaunchKernelGGL((wfp_shade_kernel<false, true>), g, b64, 0, st, c->dev, A, P, d, n, a0, a1, a2, a3, max_depth);
    else hipLaunchKernelGGL((wfp_shade_kernel<false, false>), g, b64, 0, st, c->dev, A, P, d, n, a0, a1, a2, a3, max_depth);
    RT_HIP(hipGetLastError());
    uint32_t cb[RT_WFP_COUNT + 2];        // the whole counter block in one copy: level counts, pair counts
    RT_HIP(hipMemcpyAsync(cb, A.count, sizeof cb, hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
    *next = d < max_depth ? cb[d + 1] : 0u;
    const uint32_t pc[2] = {cb[RT_WFP_COUNT], cb[RT_WFP_COUNT + 1]};
    if (pc[0] <= P.cap && pc[1] <= P.cap) return RT_OK;
    rc = wfp_arena(c, st, R, A.cap, std::max(pc[0], pc[1]), &P);   // grow (synchronises), then this level again
    if (rc) return rc;
    P.count = A.count + RT_WFP_COUNT;
    bins[0] = P.bins; bins[1] = P.bins + 4096; bins[2] = P.bins + 8192;
    if (d < max_depth) RT_HIP(hipMemsetAsync(A.count + d + 1, 0, 4, st));
  }
}

// The wavefront path (wf_*_kernel): level 0 (the pixel slots), then each level the previous one
// appended to, sorted by coherence key; then the folds, deepest level first; then the overflow
// fix-up.  The host reads every level's ray count (one stream synchronisation per level) to launch
// exactly one wave per 64 rays and to stop at the first empty level.
static int launch_wavefront(rt_ctx* c, hipStream_t st, int a0, int a1, int a2, int a3, int max_depth, uint8_t* target,
                            size_t tstride, bool f64, int rgbi, size_t n_tiles) {
  const size_t slots = n_tiles * 64, cap = std::max<size_t>(64, (slots * (size_t)c->wf_cap_pct / 100 + 63) & ~(size_t)63);
  if (cap > 0x7fffffffull || slots > 0x7fffffffull) return fail(RT_ERR_UNSUPPORTED, "wavefront launch of %zu pixel slots too large", slots);
  size_t sort_bytes = 0;
  RT_HIP(rt_wf_sort_pairs(nullptr, &sort_bytes, nullptr, nullptr, nullptr, nullptr, (int)cap, 30, st));
  const size_t levels = slots * RT_WF_BYTES0 + (size_t)max_depth * cap * RT_WF_BYTES;
  const size_t o_cnt = (levels + 255) & ~(size_t)255, o_ovf = o_cnt + 256, o_kout = (o_ovf + slots + 255) & ~(size_t)255;
  const size_t o_perm = o_kout + cap * 4, o_tmp = (o_perm + cap * 4 + 255) & ~(size_t)255, bytes = o_tmp + sort_bytes + 256;
  if (c->wf_bytes < bytes) {
    if (c->wf) (void)hipFree(c->wf);          // waits for launches that may still use it
    c->wf = nullptr;
    c->wf_bytes = 0;
    RT_HIP(hipMalloc(&c->wf, bytes));
    c->wf_bytes = bytes;
  }
  uint8_t* base = (uint8_t*)c->wf;
  WfArena A;
  A.base = base;
  A.count = (uint32_t*)(base + o_cnt);
  A.ovf = base + o_ovf;
  A.perm = nullptr;
  A.slots = (uint32_t)slots;
  A.cap = (uint32_t)cap;
  for (int k = 0; k < 3; ++k) {
    A.klo[k] = c->wf_klo[k];
    A.kscale[k] = 512.0 / std::max(1e-9, c->wf_khi[k] - c->wf_klo[k]);
  }
  uint32_t* kout = (uint32_t*)(base + o_kout);
  uint32_t* perm = (uint32_t*)(base + o_perm);
  void* tmp = base + o_tmp;
  RT_HIP(hipMemsetAsync(A.count, 0, 256, st));
  RT_HIP(hipMemsetAsync(A.ovf, 0, slots, st));
  const bool refr = c->dev.any_transparent != 0, fc = c->dev.colour_fast != 0 && c->fast_clamp;
  const bool pairs = c->wf_pairs > 0 && c->dev.shadow_pow != 0 && c->dev.n_objects > 0 && c->dev.n_objects < 4096;
  auto pairs_level = [&](int d) { return pairs && (d > 0 || c->wf_pairs == 2); };
  uint32_t n_level[RT_MAX_DEPTH_CAP + 2] = {0};
  n_level[0] = (uint32_t)slots;
  int last = 0;
  for (int d = 0; d <= max_depth; ++d) {
    const uint32_t n = n_level[d];
    if (n == 0) break;
    last = d;
    A.perm = nullptr;
    if (d > 0) {                                             // this level's slots in key order
      const WfLevel L = wf_level(A, d);                      // host-side pointer arithmetic only
      // The pair path reads a level in slot order: its candidate walks are per lane and its
      // evaluations run in object order, and the sort measured 0.3-0.6 ms per fractal frame slower
      // than none (profiles/r03o_sort_ab.txt).
      if (!pairs_level(d)) {
        size_t tb = sort_bytes;
        RT_HIP(rt_wf_sort_pairs(tmp, &tb, L.key, kout, L.val, perm, (int)n, 30, st));
        A.perm = perm;
      }
    }
    const dim3 g((n + 63) / 64);
    if (pairs_level(d)) {
      uint32_t cnt = 0;
      int rc = wfp_level(c, st, A, std::max(slots, cap), d, n, a0, a1, a2, a3, max_depth, refr, fc, &cnt);
      if (rc) return rc;
      if (d < max_depth) n_level[d + 1] = std::min<uint32_t>(cnt, (uint32_t)cap);
      continue;
    }
    else if (refr && fc) hipLaunchKernelGGL((wf_trace_kernel<true, true>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    else if (refr) hipLaunchKernelGGL((wf_trace_kernel<true, false>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    else if (fc) hipLaunchKernelGGL((wf_trace_kernel<false, true>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    else hipLaunchKernelGGL((wf_trace_kernel<false, false>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    RT_HIP(hipGetLastError());
    if (d < max_depth) {
      uint32_t cnt = 0;
      RT_HIP(hipMemcpyAsync(&cnt, A.count + d + 1, 4, hipMemcpyDeviceToHost, st));
      RT_HIP(hipStreamSynchronize(st));
      n_level[d + 1] = std::min<uint32_t>(cnt, (uint32_t)cap);
    }
  }
  const dim3 bf(256);
  for (int d = last; d >= 0; --d) {
    const uint32_t n = n_level[d];
    const dim3 gf((n + 255) / 256);
    if (f64 && fc) hipLaunchKernelGGL((wf_fold_kernel<true, true>), gf, bf, 0, st, c->dev, A, d, n, a0, a1, a2, a3, target, tstride, rgbi);
    else if (f64) hipLaunchKernelGGL((wf_fold_kernel<true, false>), gf, bf, 0, st, c->dev, A, d, n, a0, a1, a2, a3, target, tstride, rgbi);
    else if (fc) hipLaunchKernelGGL((wf_fold_kernel<false, true>), gf, bf, 0, st, c->dev, A, d, n, a0, a1, a2, a3, target, tstride, rgbi);
    else hipLaunchKernelGGL((wf_fold_kernel<false, false>), gf, bf, 0, st, c->dev, A, d, n, a0, a1, a2, a3, target, tstride, rgbi);
  }
  const dim3 gx((unsigned)c->n_cu * 4u);
#define RT_WF_FIX(R, F, FCv) hipLaunchKernelGGL((wf_fixup_kernel<R, F, FCv>), gx, dim3(64), 0, st, c->dev, A, a0, a1, a2, a3, max_depth, target, tstride, rgbi)
  if (refr && f64) { if (fc) RT_WF_FIX(true, true, true); else RT_WF_FIX(true, true, false); }
  else if (refr) { if (fc) RT_WF_FIX(true, false, true); else RT_WF_FIX(true, false, false); }
  else if (f64) { if (fc) RT_WF_FIX(false, true, true); else RT_WF_FIX(false, true, false); }
  else { if (fc) RT_WF_FIX(false, false, true); else RT_WF_FIX(false, false, false); }
#undef RT_WF_FIX
  RT_HIP(hipGetLastError());
  return RT_OK;
}

static int launch_bands(rt_ctx* c, uint32_t y_first, uint32_t band_rows, uint32_t band_pitch, uint32_t n_bands,
                        int32_t max_depth, void* out, size_t stride, void* stream, bool f64, bool rgb = false) {
  if (!c || !out) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  if (band_rows == 0 || n_bands == 0) return RT_OK;
  if (band_pitch < band_rows && n_bands > 1) return fail(RT_ERR_INVALID, "band pitch %u < band rows %u", band_pitch, band_rows);
  if (y_first >= (uint32_t)c->dev.height) return fail(RT_ERR_INVALID, "first row %u >= height %d", y_first, c->dev.height);
  const uint64_t n_rows64 = (uint64_t)band_rows * n_bands;
  if (n_rows64 > (1u << 24)) return fail(RT_ERR_INVALID, "too many rows");
  const uint32_t n_rows = (uint32_t)n_rows64;
  size_t row_bytes = (size_t)c->dev.width * (f64 ? 32 : rgb ? 3 : 4);
  const int rgbi = rgb && !f64 ? 1 : 0;
  if (stride < row_bytes) return fail(RT_ERR_INVALID, "row stride %zu < %zu", stride, row_bytes);
  if (max_depth < 0) max_depth = c->max_depth;
  if (max_depth > RT_MAX_DEPTH_CAP) return fail(RT_ERR_UNSUPPORTED, "max_depth %d > %d", max_depth, RT_MAX_DEPTH_CAP);
  RT_HIP(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;   // NULL = the device's default stream
  c->stream = st;
  const bool dev_out = is_device_ptr(out);
  uint8_t* target = (uint8_t*)out;
  size_t tstride = stride;
  if (!dev_out) {
    int rc = ensure_scratch(c, row_bytes * n_rows);
    if (rc) return rc;
    target = (uint8_t*)c->scratch;
    tstride = row_bytes;
  }
  const int tiles_x = (c->dev.width + RT_TILE_W - 1) / RT_TILE_W, tiles_y = (int)((n_rows + RT_TILE_H - 1) / RT_TILE_H);
  dim3 grid((unsigned)(tiles_x * tiles_y)), block(RT_WG_THREADS);
  const int a0 = (int)y_first, a1 = (int)band_rows, a2 = (int)band_pitch, a3 = (int)n_rows;
  // Tile order: reuse the measured order for this exact geometry, else calibrate on this launch.
  const size_t n_tiles = (size_t)tiles_x * (size_t)tiles_y;
  if (c->kernel_opt == RT_KERNEL_WAVEFRONT) {
    if (c->timing) RT_HIP(hipEventRecord(c->ev0, st));
    int rc = launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles);
    if (rc) return rc;
    if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
    c->timed = c->timing;
    if (!dev_out) {
      RT_HIP(hipMemcpy2DAsync(out, stride, target, tstride, row_bytes, n_rows, hipMemcpyDeviceToHost, st));
      RT_HIP(hipStreamSynchronize(st));
    }
    return RT_OK;
  }
  const int32_t key[7] = {a0, a1, a2, a3, max_depth, f64 ? 1 : 0, c->dev.width};
  const bool refr = c->dev.any_transparent != 0;
  // Kernel choice for scenes without a transparent object (RT_DEFERRED_MAX_TILES): the per-lane
  // megakernel is fastest when the launch fills the GPU many times over (throughput-bound); a
  // launch bound by its costliest tiles' latency takes the deferred-shadow kernel with split
  // costly tiles (DESIGN.md "Deferred shadows").  An ordered launch takes its slot's choice.
#ifdef RT_DIAG_NO_CHAIN                 // diagnostic A/B builds only: ray trees' kernel for chain scenes too
  const bool chain = false;
#else
  const bool chain = refr && c->dev.ray_chains != 0;
#endif
  // the deferred kernel takes scenes whose rays form chains (reflection-only, or refraction chains);
  // the library's own choice (AUTO) takes it for reflection-only scenes only: on refraction chains it
  // measured 3.2x slower than the chain megakernel (spinning_globes 1080p lone frame 0.80 vs 0.25 ms,
  // profiles/r03b_chain_ab.txt), so there it runs only when RT_KERNEL_DEFERRED asks for it
  const bool eligible = (!refr || chain) && c->dev.n_lights <= RT_SH_TRCAP && n_tiles <= (size_t)RT_SPLIT_TILE_MASK + 1;
  const bool auto_ok = eligible && !refr;
  // -1 auto, 0 megakernel, 1 deferred (the context's RT_OPT_KERNEL)
  const int dmode = c->kernel_opt == RT_KERNEL_MEGA ? 0 : c->kernel_opt == RT_KERNEL_DEFERRED ? 1 : -1;
  rt_ctx::OrderSlot* slot = nullptr;
  bool calibrate = false;
  if (c->tile_order && n_tiles >= RT_ORDER_MIN_TILES) {
    for (auto& s : c->order)
      if (s.valid && memcmp(s.key, key, sizeof(key)) == 0) slot = &s;
    if (!slot) {                      // calibrate into the empty or least recently used slot
      slot = &c->order[0];
      for (auto& s : c->order) {
        if (!s.valid) { slot = &s; break; }
        if (s.last_use < slot->last_use) slot = &s;
      }
      drop_order(*slot);
      RT_HIP(hipMalloc((void**)&slot->d_order, (n_tiles + 4) * sizeof(int32_t)));   // + 4: RT_DIAG_LDS_SCENE groups
      RT_HIP(hipMalloc((void**)&slot->d_cost, n_tiles * sizeof(uint32_t)));
      RT_HIP(hipMemsetAsync(slot->d_cost, 0, n_tiles * sizeof(uint32_t), st));   // tiles that store no cost sort last
      memcpy(slot->key, key, sizeof(key));
      slot->n_tiles = n_tiles;
      slot->grid = (uint32_t)n_tiles;
      calibrate = true;
    }
    slot->last_use = ++c->use_clock;
  }
  const int32_t* order = slot && !calibrate ? slot->d_order : nullptr;
  uint32_t* cost = calibrate ? slot->d_cost : nullptr;
  if (order) grid.x = slot->grid;
#ifdef RT_DIAG_LDS_SCENE
  const dim3 grid_tiles = grid;
  grid.x = (grid.x + 3) / 4;                     // 4 tiles per 256-thread workgroup (render_rows_kernel)
  block.x = 256;
  (void)grid_tiles;
#endif
  bool deferred;
  if (!eligible || dmode == 0) deferred = false;
  else if (dmode == 1) deferred = true;
  else if (!auto_ok) deferred = false;
  else if (order) deferred = slot->deferred;
  else if (calibrate) deferred = false;                       // calibrate on the megakernel
  else deferred = n_tiles < RT_ORDER_MIN_TILES || (!c->tile_order && n_tiles < RT_DEFERRED_MAX_TILES);
  if (c->timing) RT_HIP(hipEventRecord(c->ev0, st));
#define RT_LAUNCH_ROWS(R, F)                                                                                  \
  if (calibrate && fc) hipLaunchKernelGGL((render_rows_kernel<R, F, true, true>), grid, block, 0, st, c->dev, a0, a1, \
                                          a2, a3, max_depth, target, tstride, order, cost, rgbi);                       \
  else if (calibrate) hipLaunchKernelGGL((render_rows_kernel<R, F, true, false>), grid, block, 0, st, c->dev, a0, a1, \
                                         a2, a3, max_depth, target, tstride, order, cost, rgbi);                        \
  else if (fc) hipLaunchKernelGGL((render_rows_kernel<R, F, false, true>), grid, block, 0, st, c->dev, a0, a1, a2, a3, \
                                  max_depth, target, tstride, order, cost, rgbi);                                       \
  else hipLaunchKernelGGL((render_rows_kernel<R, F, false, false>), grid, block, 0, st, c->dev, a0, a1, a2, a3,   \
                          max_depth, target, tstride, order, cost, rgbi);
#ifdef RT_DIAG_ENTRY_TIMES
  if (order && deferred) {                 // diagnostic: RT_DIAG_HOT=K priority entries, RT_DIAG_GRID=K first K only
    const char* hv = getenv("RT_DIAG_HOT");
    const unsigned hot = hv ? (unsigned)atoi(hv) : 0u;
    RT_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_diag_hot), &hot, 4));
    if (const char* gv = getenv("RT_DIAG_GRID")) grid.x = std::min<unsigned>(grid.x, (unsigned)atoi(gv));
  }
#endif
#define RT_LAUNCH_DEFERRED(F, R)                                                                                \
  if (calibrate && fc) hipLaunchKernelGGL((render_rows_deferred_kernel<F, true, true, R>), grid, dim3(64), 0, st,    \
                                          c->dev, a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);     \
  else if (calibrate) hipLaunchKernelGGL((render_rows_deferred_kernel<F, true, false, R>), grid, dim3(64), 0, st,    \
                                         c->dev, a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);      \
  else if (fc) hipLaunchKernelGGL((render_rows_deferred_kernel<F, false, true, R>), grid, dim3(64), 0, st, c->dev,   \
                                  a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);                     \
  else hipLaunchKernelGGL((render_rows_deferred_kernel<F, false, false, R>), grid, dim3(64), 0, st, c->dev, a0, a1,  \
                          a2, a3, max_depth, target, tstride, order, cost, rgbi);
  const bool fc = c->dev.colour_fast != 0 && c->fast_clamp;
  // Ray-tree scenes (a transparent AND reflective object) under RT_KERNEL_AUTO: the first ordered
  // launch of a geometry is timed against one wavefront launch of the same rows, and the faster
  // path takes every later launch (fractal.scene 1080p: 16.4 vs 25.9 ms, profiles/r03d_timing.txt;
  // the small ray-tree scenes of the fuzz suite mostly keep the megakernel).  Same pixels either way.
  const bool tree = refr && !chain;
  if (order && tree && slot->wf_tune == 2) {
    int rc = launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles);
    if (rc) return rc;
    if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
    c->timed = c->timing;
    if (!dev_out) {
      RT_HIP(hipMemcpy2DAsync(out, stride, target, tstride, row_bytes, n_rows, hipMemcpyDeviceToHost, st));
      RT_HIP(hipStreamSynchronize(st));
    }
    return RT_OK;
  }
  const bool tune = order && tree && dmode == -1 && slot->wf_tune == 0;
  if (tune) RT_HIP(hipEventRecord(c->tev0, st));
  if (deferred && chain && f64) { RT_LAUNCH_DEFERRED(true, true) }
  else if (deferred && chain) { RT_LAUNCH_DEFERRED(false, true) }
  else if (chain && f64) { RT_LAUNCH_ROWS(RT_MODE_CHAIN, true) }
  else if (chain) { RT_LAUNCH_ROWS(RT_MODE_CHAIN, false) }
  else if (refr && f64) { RT_LAUNCH_ROWS(RT_MODE_TREE, true) }
  else if (refr) { RT_LAUNCH_ROWS(RT_MODE_TREE, false) }
  else if (deferred && f64) { RT_LAUNCH_DEFERRED(true, false) }
  else if (deferred) { RT_LAUNCH_DEFERRED(false, false) }
  else if (f64) { RT_LAUNCH_ROWS(RT_MODE_REFL, true) }
  else { RT_LAUNCH_ROWS(RT_MODE_REFL, false) }
#undef RT_LAUNCH_ROWS
#undef RT_LAUNCH_DEFERRED
  RT_HIP(hipGetLastError());
  if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
  c->timed = c->timing;
  if (tune) {                         // synchronous, once per ray-tree geometry (see above)
    float mega_ms = 0.0f, wf_ms = 0.0f;
    RT_HIP(hipEventRecord(c->tev1, st));
    RT_HIP(hipEventSynchronize(c->tev1));
    RT_HIP(hipEventElapsedTime(&mega_ms, c->tev0, c->tev1));
    RT_HIP(hipEventRecord(c->tev0, st));
    int rc = launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles);
    if (rc) return rc;
    RT_HIP(hipEventRecord(c->tev1, st));
    RT_HIP(hipEventSynchronize(c->tev1));
    RT_HIP(hipEventElapsedTime(&wf_ms, c->tev0, c->tev1));
    slot->wf_tune = wf_ms < mega_ms ? 2 : 1;
    static const bool order_debug = getenv("RT_TILE_ORDER_DEBUG") != nullptr;
    if (order_debug)
      fprintf(stderr, "ray-tree autotune: megakernel %.3f ms, wavefront %.3f ms -> %s\n", mega_ms, wf_ms,
              slot->wf_tune == 2 ? "wavefront" : "megakernel");
  }
  if (calibrate) {                    // synchronous, once per geometry and scene upload
    std::vector<uint32_t> h_cost(n_tiles);
    std::vector<int32_t> h_order(n_tiles);
    RT_HIP(hipMemcpyAsync(h_cost.data(), slot->d_cost, n_tiles * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
    // Longest-first: every tile placed by its own measured cost (runs of 2-30 neighbouring tiles
    // sorted together, zigzag and partly row-major orders measured 3-60 % slower,
    // profiles/r01ah_tile_order_sweep.txt, r02k_order_ab.txt).
    for (size_t i = 0; i < n_tiles; ++i) h_order[i] = (int32_t)i;
    std::stable_sort(h_order.begin(), h_order.end(), [&](int32_t x, int32_t y) { return h_cost[x] > h_cost[y]; });
    bool tail_bound = false;
    // wave slots of the calibrated (mega)kernel on this device
    const double slots = (double)c->n_cu * 4.0 * (double)(!refr ? RT_WAVES_PER_EU_NOREFR : c->dev.ray_chains ? RT_WAVES_PER_EU_CHAIN : RT_WAVES_PER_EU);
    if (auto_ok && dmode == -1 && n_tiles < RT_DEFERRED_MAX_TILES) {
      uint64_t sum = 0, mx = 0;
      for (uint32_t v : h_cost) { sum += v; mx = v > mx ? v : mx; }
      tail_bound = (double)mx > (double)sum / slots;
    }
    slot->deferred = eligible && (dmode == 1 || tail_bound);
    if (slot->deferred) {
      // Split the costliest tiles over P = 2, 4 or 8 waves (cost >= k * P * the median tile):
      // their shadow rays then spread over P x 64 lanes.  The factor k: 1 below 24000 tiles, 1.5
      // above.  Swept at 1 / 1.25 / 1.5 / 2 / 3
      // (profiles/r02bo_split_sweep.txt): the 4K N = 8 share (16320 tiles) 0.150 / 0.152 / 0.172 /
      // 0.170 / 0.183 ms; the N = 4 share (32400 tiles) 0.209 / 0.192 / 0.190 / 0.200 / 0.232 ms;
      // the whole 1080p d5 frame (32400 tiles) 0.208 / 0.189 / 0.184 / 0.181 / 0.225 ms.
      double split_k = n_tiles < 24000 ? 1.0 : 1.5;
#ifdef RT_DIAG_ENTRY_TIMES
      if (const char* kv = getenv("RT_DIAG_SPLIT_K")) split_k = atof(kv);
#endif
      std::vector<uint32_t> sorted_cost(h_cost);
      std::nth_element(sorted_cost.begin(), sorted_cost.begin() + n_tiles / 2, sorted_cost.end());
      const double med = std::max(1.0, (double)sorted_cost[n_tiles / 2]);
      std::vector<int32_t> split;
      split.reserve(n_tiles + n_tiles / 8);
      for (size_t i = 0; i < n_tiles; ++i) {
        const uint32_t t = (uint32_t)h_order[i];
        int lp = 0;
        while (lp < RT_SPLIT_MAX_LOG2 && h_cost[t] >= split_k * med * (double)(2 << lp)) ++lp;
        for (int part = 0; part < (1 << lp); ++part)
          split.push_back((int32_t)(t | ((uint32_t)part << 20) | ((uint32_t)lp << 24)));
      }
      if (split.size() > n_tiles) {
        int32_t* d = nullptr;
        RT_HIP(hipMalloc((void**)&d, split.size() * sizeof(int32_t)));
        (void)hipFree(slot->d_order);
        slot->d_order = d;
        h_order.swap(split);
      }
    }
    slot->grid = (uint32_t)h_order.size();
#ifdef RT_DIAG_LDS_SCENE
    if (!slot->deferred) h_order.resize(h_order.size() + 4, -1);   // entries past the last tile: no tile
#endif
    RT_HIP(hipMemcpyAsync(slot->d_order, h_order.data(), h_order.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    RT_HIP(hipStreamSynchronize(st));
    slot->valid = true;
    static const bool order_debug = getenv("RT_TILE_ORDER_DEBUG") != nullptr;
    if (order_debug) {                      // wave times in wall-clock ticks (100 MHz)
      std::vector<uint32_t> v(h_cost);
      std::sort(v.begin(), v.end());
      double sum = 0.0;
      for (uint32_t x : v) sum += x;
      fprintf(stderr, "tile order: %zu tiles, max %u, p99 %u, p90 %u, median %u, mean %.1f ticks; max / (sum / %.0f slots) = %.3f; "
              "ordered launches: %s kernel, %u entries\n", n_tiles, v.back(), v[n_tiles * 99 / 100], v[n_tiles * 9 / 10],
              v[n_tiles / 2], sum / n_tiles, slots, v.back() / (sum / slots), slot->deferred ? "deferred" : "mega", slot->grid);
    }
  }
  if (!dev_out) {
    RT_HIP(hipMemcpy2DAsync(out, stride, target, tstride, row_bytes, n_rows, hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
  }
  return RT_OK;
}

static int launch_rows(rt_ctx* c, uint32_t y0, uint32_t y1, int32_t max_depth, void* out, size_t stride,
                       void* stream, bool f64) {
  if (!c || !out) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  if (y0 > y1 || y1 > (uint32_t)c->dev.height) return fail(RT_ERR_INVALID, "bad row range [%u, %u) for height %d", y0, y1, c->dev.height);
  if (y0 == y1) return RT_OK;
  return launch_bands(c, y0, y1 - y0, y1 - y0, 1, max_depth, out, stride, stream, f64);
}

int rt_render_row_bands(rt_ctx* c, uint32_t y_first, uint32_t band_rows, uint32_t band_pitch, uint32_t n_bands,
                        int32_t max_depth, uint8_t* rgba8, size_t row_stride_bytes, void* stream) {
  return launch_bands(c, y_first, band_rows, band_pitch, n_bands, max_depth, rgba8, row_stride_bytes, stream, false);
}

int rt_render_row_bands_rgb8(rt_ctx* c, uint32_t y_first, uint32_t band_rows, uint32_t band_pitch, uint32_t n_bands,
                             int32_t max_depth, uint8_t* rgb8, size_t row_stride_bytes, void* stream) {
  return launch_bands(c, y_first, band_rows, band_pitch, n_bands, max_depth, rgb8, row_stride_bytes, stream, false, true);
}

int rt_render_rows(rt_ctx* c, uint32_t y0, uint32_t y1, int32_t max_depth, uint8_t* rgba8,
                   size_t row_stride_bytes, void* stream) {
  return launch_rows(c, y0, y1, max_depth, rgba8, row_stride_bytes, stream, false);
}

int rt_render_rows_f64(rt_ctx* c, uint32_t y0, uint32_t y1, int32_t max_depth, double* rgba,
                       size_t row_stride_bytes, void* stream) {
  return launch_rows(c, y0, y1, max_depth, rgba, row_stride_bytes, stream, true);
}

int rt_assemble_row_bands(const uint8_t* gathered, size_t gathered_stride, uint32_t world, uint32_t slot_rows,
                          uint32_t band_rows, uint32_t height, size_t row_bytes, uint8_t* frame, size_t frame_stride,
                          void* stream) {
  if (!gathered || !frame) return fail(RT_ERR_INVALID, "null argument");
  if (world == 0 || band_rows == 0) return fail(RT_ERR_INVALID, "world and band_rows must be > 0");
  if (height == 0 || row_bytes == 0) return RT_OK;
  if (height > (1u << 24)) return fail(RT_ERR_INVALID, "too many rows");
  const uint64_t bands = ((uint64_t)height + band_rows - 1) / band_rows, per_rank = (bands + world - 1) / world;
  if ((uint64_t)slot_rows < per_rank * band_rows)
    return fail(RT_ERR_INVALID, "slot of %u rows holds fewer than %llu bands of %u rows", slot_rows,
                (unsigned long long)per_rank, band_rows);
  if (slot_rows > (1u << 24) || (uint64_t)slot_rows * world > (1u << 30)) return fail(RT_ERR_INVALID, "slot too large");
  if (gathered_stride < row_bytes || frame_stride < row_bytes) return fail(RT_ERR_INVALID, "row stride < row bytes");
  if (!is_device_ptr(gathered) || !is_device_ptr(frame)) return fail(RT_ERR_INVALID, "frame assembly takes device pointers");
  const bool v16 = (((uintptr_t)gathered | (uintptr_t)frame | gathered_stride | frame_stride | row_bytes) & 15) == 0;
  hipLaunchKernelGGL(assemble_bands_kernel, dim3(height), dim3(256), 0, (hipStream_t)stream, gathered, gathered_stride,
                     (int)world, (int)slot_rows, (int)band_rows, row_bytes, frame, frame_stride, v16 ? 1 : 0);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

int rt_assemble_row_bands_rgb8(const uint8_t* gathered, size_t gathered_stride, uint32_t world, uint32_t slot_rows,
                               uint32_t band_rows, uint32_t height, uint32_t width, uint8_t* frame, size_t frame_stride,
                               void* stream) {
  if (!gathered || !frame) return fail(RT_ERR_INVALID, "null argument");
  if (world == 0 || band_rows == 0) return fail(RT_ERR_INVALID, "world and band_rows must be > 0");
  if (height == 0 || width == 0) return RT_OK;
  if (height > (1u << 24) || width > (1u << 24)) return fail(RT_ERR_INVALID, "frame too large");
  const uint64_t bands = ((uint64_t)height + band_rows - 1) / band_rows, per_rank = (bands + world - 1) / world;
  if ((uint64_t)slot_rows < per_rank * band_rows)
    return fail(RT_ERR_INVALID, "slot of %u rows holds fewer than %llu bands of %u rows", slot_rows,
                (unsigned long long)per_rank, band_rows);
  if (slot_rows > (1u << 24) || (uint64_t)slot_rows * world > (1u << 30)) return fail(RT_ERR_INVALID, "slot too large");
  if (gathered_stride < (size_t)width * 3 || frame_stride < (size_t)width * 4) return fail(RT_ERR_INVALID, "row stride < row bytes");
  if ((((uintptr_t)frame) | frame_stride) & 3) return fail(RT_ERR_INVALID, "frame rows must be 4-byte aligned");
  if (!is_device_ptr(gathered) || !is_device_ptr(frame)) return fail(RT_ERR_INVALID, "frame assembly takes device pointers");
  const bool vec = (width & 3) == 0 && (((uintptr_t)gathered | gathered_stride) & 3) == 0 &&
                   (((uintptr_t)frame | frame_stride) & 15) == 0;
  hipLaunchKernelGGL(assemble_bands_rgb_kernel, dim3(height), dim3(256), 0, (hipStream_t)stream, gathered, gathered_stride,
                     (int)world, (int)slot_rows, (int)band_rows, (int)width, frame, frame_stride, vec ? 1 : 0);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

// antialiaser.rs:87-191 over a whole quantised frame (see the kernels above).
int rt_antialias(rt_ctx* c, const uint8_t* src_rgba8, size_t src_stride, double threshold, int32_t level,
                 int32_t max_depth, uint8_t* dst_rgba8, size_t dst_stride, double* dst_f64, size_t f64_stride,
                 uint64_t* rays_traced, void* stream) {
  if (!c || !src_rgba8 || (!dst_rgba8 && !dst_f64)) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  if (level < 0) level = 0;
  if (level > RT_AA_MAX_LEVEL) return fail(RT_ERR_UNSUPPORTED, "anti-aliasing level %d > %d", level, RT_AA_MAX_LEVEL);
  if (!(threshold == threshold)) return fail(RT_ERR_INVALID, "threshold is NaN");
  if (max_depth < 0) max_depth = c->max_depth;
  if (max_depth > RT_MAX_DEPTH_CAP) return fail(RT_ERR_UNSUPPORTED, "max_depth %d > %d", max_depth, RT_MAX_DEPTH_CAP);
  const int W = c->dev.width, H = c->dev.height;
  if (W > 65535 || H > 65535) return fail(RT_ERR_UNSUPPORTED, "frame %dx%d too large for the edge list", W, H);
  const size_t row4 = (size_t)W * 4, row32 = (size_t)W * 32;
  if (src_stride < row4) return fail(RT_ERR_INVALID, "source stride %zu < %zu", src_stride, row4);
  if (dst_rgba8 && dst_stride < row4) return fail(RT_ERR_INVALID, "output stride %zu < %zu", dst_stride, row4);
  if (dst_f64 && f64_stride < row32) return fail(RT_ERR_INVALID, "f64 stride %zu < %zu", f64_stride, row32);
  RT_HIP(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  c->stream = st;
  const size_t npx = (size_t)W * H;
  // device staging: [src u8][dst u8][dst f64][edges][counters] for host pointers
  const bool d_src = is_device_ptr(src_rgba8), d_u8 = !dst_rgba8 || is_device_ptr(dst_rgba8);
  const bool d_f64 = !dst_f64 || is_device_ptr(dst_f64);
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = (off + bytes + 255) & ~(size_t)255; return o; };
  const size_t o_src = d_src ? 0 : take(npx * 4), o_u8 = d_u8 ? 0 : take(npx * 4), o_f64 = d_f64 ? 0 : take(npx * 32);
  const size_t o_edges = take(npx * 4), o_cnt = take(64);
  int rc = ensure_scratch(c, off);
  if (rc) return rc;
  uint8_t* sb = (uint8_t*)c->scratch;
  const uint8_t* src = d_src ? src_rgba8 : sb + o_src;
  size_t sstride = src_stride;
  if (!d_src) { RT_HIP(hipMemcpy2DAsync(sb + o_src, row4, src_rgba8, src_stride, row4, H, hipMemcpyHostToDevice, st)); sstride = row4; }
  uint8_t* u8 = dst_rgba8 ? (d_u8 ? dst_rgba8 : sb + o_u8) : nullptr;
  size_t u8s = d_u8 ? dst_stride : row4;
  double* f64 = dst_f64 ? (d_f64 ? dst_f64 : (double*)(sb + o_f64)) : nullptr;
  size_t f64s = d_f64 ? f64_stride : row32;
  uint32_t* edges = (uint32_t*)(sb + o_edges);
  uint32_t* cnt = (uint32_t*)(sb + o_cnt);
  RT_HIP(hipMemsetAsync(cnt, 0, 64, st));
  if (c->timing) RT_HIP(hipEventRecord(c->ev0, st));
  const int tiles = ((W + 15) / 16) * ((H + 15) / 16);
  hipLaunchKernelGGL(aa_classify_kernel, dim3(tiles), dim3(256), 0, st, src, sstride, W, H, threshold, (int)level,
                     u8, u8s, f64, f64s, edges, cnt);
  RT_HIP(hipGetLastError());
  uint32_t n_edges = 0;
  RT_HIP(hipMemcpyAsync(&n_edges, cnt, 4, hipMemcpyDeviceToHost, st));
  RT_HIP(hipStreamSynchronize(st));
  uint64_t rays = 0;
  if (n_edges > 0) {
    const int sz = (1 << level) + 1;
    const size_t per_col = (size_t)sz * sz * sizeof(AaCol), per_have = RT_AA_HAVE_WORDS * 8;
    size_t max_new = 0;                                           // largest pass: (2^p+1)^2 - (2^(p-1)+1)^2
    for (int p = 1; p <= level; ++p) {
      size_t a = ((size_t)1 << p) + 1, b = ((size_t)1 << (p - 1)) + 1;
      max_new = a * a - b * b > max_new ? a * a - b * b : max_new;
    }
    const size_t cap = (size_t)n_edges * max_new;
    if (cap > 0xffffffffull) return fail(RT_ERR_UNSUPPORTED, "too many anti-aliasing samples");
    void* work = nullptr;
    const size_t bytes = (size_t)n_edges * (per_col + per_have) + cap * sizeof(uint2) + 256;
    RT_HIP(hipMallocAsync(&work, bytes, st));
    AaGrid G;
    G.col = (AaCol*)work;
    G.have = (uint64_t*)((uint8_t*)work + (size_t)n_edges * per_col);
    G.size = sz;
    uint2* req = (uint2*)((uint8_t*)G.have + (size_t)n_edges * per_have);
    const dim3 eg((n_edges + 255) / 256), blk(256);
    hipLaunchKernelGGL(aa_init_kernel, eg, blk, 0, st, G, src, sstride, edges, n_edges);
    int err = RT_OK;
    for (int pass = 1; pass <= level && err == RT_OK; ++pass) {
      if (hipMemsetAsync(cnt + 1, 0, 4, st) != hipSuccess) { err = fail(RT_ERR_DEVICE, "memset failed"); break; }
      hipLaunchKernelGGL(aa_expand_kernel, eg, blk, 0, st, G, n_edges, pass, (int)level, threshold, req, cnt + 1, (uint32_t)cap);
      uint32_t n_req = 0;
      if (hipMemcpyAsync(&n_req, cnt + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) { err = fail(RT_ERR_DEVICE, "anti-aliasing expand failed"); break; }
      if (n_req > cap) { err = fail(RT_ERR_DEVICE, "anti-aliasing request overflow (%u > %zu)", n_req, cap); break; }
      if (n_req == 0) break;
      rays += n_req;
      const dim3 rg((n_req + 63) / 64);
      const bool fc = c->dev.colour_fast != 0 && c->fast_clamp;
#define RT_LAUNCH_AA(R, F) hipLaunchKernelGGL((aa_trace_kernel<R, F>), rg, dim3(64), 0, st, c->dev, G, edges, req, n_req, (int)max_depth)
      if (c->dev.any_transparent && fc) RT_LAUNCH_AA(true, true);
      else if (c->dev.any_transparent) RT_LAUNCH_AA(true, false);
      else if (fc) RT_LAUNCH_AA(false, true);
      else RT_LAUNCH_AA(false, false);
#undef RT_LAUNCH_AA
    }
    if (err == RT_OK) {
      hipLaunchKernelGGL(aa_resolve_kernel, eg, blk, 0, st, G, edges, n_edges, (int)level, threshold, u8, u8s, f64, f64s);
      if (hipGetLastError() != hipSuccess) err = fail(RT_ERR_DEVICE, "anti-aliasing kernels failed to launch");
    }
    (void)hipFreeAsync(work, st);
    if (err) return err;
  }
  if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
  c->timed = c->timing;
  if (dst_rgba8 && !d_u8) RT_HIP(hipMemcpy2DAsync(dst_rgba8, dst_stride, u8, row4, row4, H, hipMemcpyDeviceToHost, st));
  if (dst_f64 && !d_f64) RT_HIP(hipMemcpy2DAsync(dst_f64, f64_stride, f64, row32, row32, H, hipMemcpyDeviceToHost, st));
  RT_HIP(hipStreamSynchronize(st));
  if (rays_traced) *rays_traced = rays;
  return RT_OK;
}

// debug_window.rs:166-227 for rows [y0, y1) of the scene's frame size.
int rt_render_ortho(rt_ctx* c, int32_t axis1, int32_t axis2, double dir1, double dir2, double scale, uint32_t y0,
                    uint32_t y1, uint8_t* rgba8, size_t row_stride_bytes, double* rgba_f64, size_t f64_stride,
                    void* stream) {
  if (!c || (!rgba8 && !rgba_f64)) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  OrthoView V;
  if (axis1 < 0 || axis1 > 2 || axis2 < 0 || axis2 > 2) return fail(RT_ERR_INVALID, "Invalid axes");
  if (axis1 != 0 && axis2 != 0) V.axis3 = 0;
  else if (axis1 != 1 && axis2 != 1) V.axis3 = 1;
  else if (axis1 != 2 && axis2 != 2) V.axis3 = 2;
  else return fail(RT_ERR_INVALID, "Invalid axes");                      // the reference panics
  V.axis1 = axis1; V.axis2 = axis2; V.dir1 = dir1; V.dir2 = dir2; V.scale = scale;
  if (y0 > y1 || y1 > (uint32_t)c->dev.height) return fail(RT_ERR_INVALID, "bad row range [%u, %u)", y0, y1);
  if (y0 == y1) return RT_OK;
  const int W = c->dev.width;
  const uint32_t n = y1 - y0;
  const size_t row4 = (size_t)W * 4, row32 = (size_t)W * 32;
  if (rgba8 && row_stride_bytes < row4) return fail(RT_ERR_INVALID, "row stride %zu < %zu", row_stride_bytes, row4);
  if (rgba_f64 && f64_stride < row32) return fail(RT_ERR_INVALID, "f64 stride %zu < %zu", f64_stride, row32);
  RT_HIP(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  c->stream = st;
  const bool d8 = !rgba8 || is_device_ptr(rgba8), df = !rgba_f64 || is_device_ptr(rgba_f64);
  uint8_t* t8 = rgba8;
  double* tf = rgba_f64;
  size_t s8 = row_stride_bytes, sf = f64_stride;
  if (!d8 || !df) {
    int rc = ensure_scratch(c, (d8 ? 0 : row4 * n) + (df ? 0 : row32 * n) + 256);
    if (rc) return rc;
    uint8_t* sb = (uint8_t*)c->scratch;
    if (!d8) { t8 = sb; s8 = row4; sb += (row4 * n + 255) & ~(size_t)255; }
    if (!df) { tf = (double*)sb; sf = row32; }
  }
  const int tiles = ((W + 15) / 16) * (int)((n + 15) / 16);
  if (c->timing) RT_HIP(hipEventRecord(c->ev0, st));
  hipLaunchKernelGGL(ortho_kernel, dim3(tiles), dim3(256), 0, st, c->dev, V, (int)y0, (int)n, t8, s8, tf, sf);
  RT_HIP(hipGetLastError());
  if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
  c->timed = c->timing;
  if (!d8) RT_HIP(hipMemcpy2DAsync(rgba8, row_stride_bytes, t8, row4, row4, n, hipMemcpyDeviceToHost, st));
  if (!df) RT_HIP(hipMemcpy2DAsync(rgba_f64, f64_stride, tf, row32, row32, n, hipMemcpyDeviceToHost, st));
  if (!d8 || !df) RT_HIP(hipStreamSynchronize(st));
  return RT_OK;
}

// RayDebugger::record_rays (ray_debugger.rs:92-137): one thread, records in callback order.
int rt_record_rays(rt_ctx* c, double x, double y, int32_t max_depth, rt_ray_record* records, int32_t cap,
                   int32_t* n_rays, double* rgba) {
  if (!c || (!records && cap > 0) || cap < 0 || !n_rays) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  if (max_depth < 0) max_depth = c->max_depth;
  if (max_depth > RT_MAX_DEPTH_CAP) return fail(RT_ERR_UNSUPPORTED, "max_depth %d > %d", max_depth, RT_MAX_DEPTH_CAP);
  RT_HIP(hipSetDevice(c->device));
  // room for the whole ray tree: a chain of max_depth + 1 rays, or a binary tree with refraction
  const bool refr = c->dev.any_transparent != 0;
  const int dev_cap = refr ? (2 << max_depth) - 1 : max_depth + 1;
  const size_t rec_bytes = sizeof(rt_ray_record) * ((size_t)dev_cap + 1);
  const size_t ord_off = (rec_bytes + 255) & ~(size_t)255, cnt_off = ord_off + (((size_t)dev_cap * 4 + 255) & ~(size_t)255);
  int rc = ensure_scratch(c, cnt_off + 64);
  if (rc) return rc;
  uint8_t* sb = (uint8_t*)c->scratch;
  rt_ray_record* d_rec = (rt_ray_record*)sb;
  int* d_ord = (int*)(sb + ord_off);
  int* d_cnt = (int*)(sb + cnt_off);
  hipStream_t st = nullptr;
  c->stream = st;
  if (refr)
    hipLaunchKernelGGL((record_ray_kernel<true>), dim3(1), dim3(64), 0, st, c->dev, x, y, (int)max_depth, d_rec, d_ord, dev_cap, d_cnt);
  else
    hipLaunchKernelGGL((record_ray_kernel<false>), dim3(1), dim3(64), 0, st, c->dev, x, y, (int)max_depth, d_rec, d_ord, dev_cap, d_cnt);
  RT_HIP(hipGetLastError());
  int cnt[2] = {0, 0};
  RT_HIP(hipMemcpy(cnt, d_cnt, sizeof cnt, hipMemcpyDeviceToHost));
  if (cnt[0] != cnt[1] || cnt[1] > dev_cap) return fail(RT_ERR_DEVICE, "ray recorder overflow (%d/%d of %d)", cnt[0], cnt[1], dev_cap);
  std::vector<rt_ray_record> rec((size_t)dev_cap + 1);
  std::vector<int> ord((size_t)dev_cap);
  RT_HIP(hipMemcpy(rec.data(), d_rec, rec_bytes, hipMemcpyDeviceToHost));
  RT_HIP(hipMemcpy(ord.data(), d_ord, sizeof(int) * (size_t)dev_cap, hipMemcpyDeviceToHost));
  *n_rays = cnt[1];
  const int keep = cnt[1] < cap ? cnt[1] : cap;
  for (int i = 0; i < keep; ++i) records[i] = rec[(size_t)ord[i]];
  if (rgba) for (int k = 0; k < 4; ++k) rgba[k] = rec[(size_t)dev_cap].color[k];
  return RT_OK;
}

int rt_trace_pixel_f64(const rt_scene* scene, double x, double y, int32_t max_depth, int device, double rgba[4]) {
  if (!scene || !rgba) return fail(RT_ERR_INVALID, "null argument");
  struct Holder {                       // the calling thread's context, freed with the thread
    rt_ctx* c = nullptr;
    ~Holder() { if (c) rt_ctx_free(c); }
  };
  static thread_local Holder h;
  if (h.c && h.c->device != device) {
    rt_ctx_free(h.c);
    h.c = nullptr;
  }
  if (!h.c) {
    int rc = rt_ctx_create(device, &h.c);
    if (rc) return rc;
    rt_ctx_set_option(h.c, RT_OPT_TIMING, 0);
  }
  int rc = rt_ctx_upload(h.c, scene);
  if (rc) return rc;
  const double xy[2] = {x, y};
  return rt_render_points_f64(h.c, xy, 1, max_depth, rgba, nullptr);
}

int rt_render_points_f64(rt_ctx* c, const double* xy, size_t n, int32_t max_depth, double* out, void* stream) {
  if (!c || !xy || !out) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  if (max_depth < 0) max_depth = c->max_depth;
  if (max_depth > RT_MAX_DEPTH_CAP) return fail(RT_ERR_UNSUPPORTED, "max_depth %d > %d", max_depth, RT_MAX_DEPTH_CAP);
  if (n == 0) return RT_OK;
  RT_HIP(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;   // NULL = the device's default stream
  c->stream = st;
  const bool dev_in = is_device_ptr(xy), dev_out = is_device_ptr(out);
  const double* in = xy;
  double* target = out;
  if (!dev_in || !dev_out) {
    int rc = ensure_scratch(c, n * 6 * sizeof(double));
    if (rc) return rc;
    double* sx = (double*)c->scratch;
    if (!dev_in) { RT_HIP(hipMemcpyAsync(sx, xy, n * 2 * sizeof(double), hipMemcpyHostToDevice, st)); in = sx; }
    if (!dev_out) target = sx + 2 * n;
  }
  dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (c->timing) RT_HIP(hipEventRecord(c->ev0, st));
  if (c->dev.any_transparent) hipLaunchKernelGGL((render_points_kernel<true>), grid, block, 0, st, c->dev, in, n, max_depth, target);
  else hipLaunchKernelGGL((render_points_kernel<false>), grid, block, 0, st, c->dev, in, n, max_depth, target);
  RT_HIP(hipGetLastError());
  if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
  c->timed = c->timing;
  if (!dev_out) {
    RT_HIP(hipMemcpyAsync(out, target, n * 4 * sizeof(double), hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
  }
  return RT_OK;
}

int rt_ctx_last_kernel_ms(rt_ctx* c, float* ms) {
  if (!c || !ms) return fail(RT_ERR_INVALID, "null argument");
  if (!c->timed) return fail(RT_ERR_INVALID, c->timing ? "no launch recorded" : "RT_OPT_TIMING is off");
  RT_HIP(hipEventSynchronize(c->ev1));
  RT_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
  return RT_OK;
}

int rt_ctx_set_option(rt_ctx* c, int32_t option, int32_t value) {
  if (!c) return fail(RT_ERR_INVALID, "null context");
  if (option == RT_OPT_TIMING) {
    if (value != 0 && value != 1) return fail(RT_ERR_INVALID, "RT_OPT_TIMING value %d", value);
    c->timing = value != 0;
    c->timed = false;                  // no launch recorded under the new setting yet
    return RT_OK;
  }
  if (option == RT_OPT_WAVEFRONT_PAIRS) {
    if (value < 0 || value > 2) return fail(RT_ERR_INVALID, "RT_OPT_WAVEFRONT_PAIRS %d not in [0, 2]", value);
    c->wf_pairs = value;
    return RT_OK;
  }
  if (option == RT_OPT_WAVEFRONT_CAP) {
    if (value < 1 || value > 400) return fail(RT_ERR_INVALID, "RT_OPT_WAVEFRONT_CAP %d not in [1, 400]", value);
    c->wf_cap_pct = value;
    return RT_OK;
  }
  if (option == RT_OPT_TILE_ORDER || option == RT_OPT_FAST_CLAMP) {
    if (value != 0 && value != 1) return fail(RT_ERR_INVALID, "option %d value %d", option, value);
    if (option == RT_OPT_FAST_CLAMP) {
      c->fast_clamp = value != 0;
    } else if (c->tile_order != (value != 0)) {
      RT_HIP(hipSetDevice(c->device));
      drop_orders(c);
      c->tile_order = value != 0;
    }
    return RT_OK;
  }
  if (option != RT_OPT_KERNEL) return fail(RT_ERR_INVALID, "unknown option %d", option);
  if (value != RT_KERNEL_AUTO && value != RT_KERNEL_MEGA && value != RT_KERNEL_DEFERRED && value != RT_KERNEL_WAVEFRONT)
    return fail(RT_ERR_INVALID, "RT_OPT_KERNEL value %d", value);
  if (value != c->kernel_opt) {
    // tile orders were built for one kernel (split entries only for the deferred one): rebuild
    RT_HIP(hipSetDevice(c->device));
    drop_orders(c);
    c->kernel_opt = value;
  }
  return RT_OK;
}

int rt_stream_create(int device, void** stream) {
  if (!stream) return fail(RT_ERR_INVALID, "null argument");
  int n_dev = 0;
  RT_HIP(hipGetDeviceCount(&n_dev));
  if (device < 0 || device >= n_dev) return fail(RT_ERR_INVALID, "device %d of %d", device, n_dev);
  RT_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  RT_HIP(hipGetDeviceProperties(&prop, device));
  // every CU enabled: the mask only buys the stream a hardware queue of its own
  std::vector<uint32_t> mask((size_t)(prop.multiProcessorCount + 31) / 32, 0xFFFFFFFFu);
  if (prop.multiProcessorCount % 32) mask.back() = (1u << (prop.multiProcessorCount % 32)) - 1u;
  hipStream_t st = nullptr;
  RT_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
  *stream = st;
  return RT_OK;
}

int rt_stream_destroy(void* stream) {
  if (!stream) return fail(RT_ERR_INVALID, "null stream");
  RT_HIP(hipStreamDestroy((hipStream_t)stream));
  return RT_OK;
}

int rt_ctx_synchronize(rt_ctx* c) {
  if (!c) return fail(RT_ERR_INVALID, "null context");
  RT_HIP(hipSetDevice(c->device));
  RT_HIP(hipStreamSynchronize(c->stream));
  return RT_OK;
}

void rt_ctx_free(rt_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->d_blob) (void)hipFree(c->d_blob);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->wf) (void)hipFree(c->wf);
  if (c->wfr) (void)hipFree(c->wfr);
  if (c->wfp) (void)hipFree(c->wfp);
  drop_orders(c);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->tev0) (void)hipEventDestroy(c->tev0);
  if (c->tev1) (void)hipEventDestroy(c->tev1);
  delete c;
}

}  // extern "C"
