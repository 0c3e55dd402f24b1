// rt_device.h -- the gfx950 (MI355X, CDNA4) device core of the TinyRaytracer render path: the
// reference's per-ray algorithm (get_ray_color and everything it calls) as device functions, shared
// by every kernel translation unit (k_rows.hip, k_wavefront.hip, k_views.hip) and by the
// scene-specialised kernel that hipRTC compiles at scene upload (k_spec.hip, RT_SPEC below).
//
// One thread per pixel; each 64-lane wave owns an 8x8 pixel tile (coherent primary rays,
// fewer divergent CSG/shade branches than a 64x1 row strip).  All arithmetic is IEEE f64 with NO
// contraction (Rust never fuses): every TU is compiled with -ffp-contract=off and the pragma
// below.  sqrt and division lower to correctly rounded sequences on gfx950 (verified bit-exact
// against glibc, profiles/r01_libm_probe.txt); acos is rt_acos (rt_math.h: 1 ulp from glibc on
// ~0.4% of inputs, and far fewer registers than ocml's); sin comes from ocml and may differ from
// glibc by 1 ulp (DESIGN.md "Parity").
//
// The reference's recursion (get_ray_color calling itself for refraction and reflection,
// raytracer.rs:242-280) becomes an explicit per-lane frame stack combined in the same
// post-order: child colour C folds into its parent as in_range(A + in_range(C * w)) where
// A = parent.intensify(1 - w) -- exactly the `final.intensify(1-w) + R.intensify(w)` of
// raytracer.rs:256-257 / :278-279.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include "../../include/rt_abi.h"
#else                                // hipRTC (spec.hip): no libc headers
#define INFINITY __builtin_inf()
using __hip_internal::size_t;
#endif

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

#pragma clang fp contract(off)

// The device functions below are inlined into every kernel.  In the specialised program (RT_SPEC,
// one module holding 8 kernels of one scene) the inliner would otherwise keep the big ones as
// calls (14 s_swappc, the call ABI's saves and scratch); every kernel instantiates its own copy.
#ifdef RT_SPEC
// A value the optimiser must treat as computed here: trace()'s light loop calls the shadow walk with
// the same origin for every light (and the shading inputs once, inside the loop), and with every box
// and transform a constant the terms on the hit point ((lo - o), xf(inv, o), every object's CSG
// inside / on-surface tests) become loop-invariant -- LICM hoists (speculates) those of EVERY box,
// leaf and object out of the light loop and the spec kernel spills ~200 VGPRs.  Re-defining the point
// where it is used keeps each term where the generic kernel computes it (no instruction, no value
// change).
#define RT_OPAQUE(x) asm volatile("" : "+v"(x))
#define RT_FN __device__ __attribute__((always_inline))
#define RT_SPEC_UNROLL _Pragma("unroll")   // loops over a constant record's runs: unroll them fully
#else
#define RT_OPAQUE(x) (void)0
#define RT_FN __device__
#define RT_SPEC_UNROLL
#endif

namespace {

// Scene tables are read-only for the whole launch: view them through the CONSTANT address space
// (4) so uniform-index reads compile to scalar (SMEM) loads instead of per-lane VMEM loads.
// A family program (RT_SPEC_FAMILY) reads its tables through generic pointers (fam_rec).
#if defined(RT_SPEC_FAMILY)
#define CAS
#else
#define CAS __attribute__((address_space(4)))
#endif
template <class T> using cptr = const CAS T*;
template <class T> __device__ __forceinline__ cptr<T> as_const(const T* p) { return (cptr<T>)p; }

// Record I of scene table `tab` (objects, trav, strav, leaves, lights) as `cptr<T> NAME`.
// RT_SPEC_FAMILY (spec.hip: ONE program for a family of scenes of the same structure -- the frames of
// an animation): the record is assembled word by word, the 4-byte words every member of the family
// shares from the program's constexpr table (they fold like the single-scene program's), the words
// that differ between members from this scene's table in HBM (scalar loads).  The table stays
// exactly the scene's own: the merge only decides which words the compiler may treat as constants.
#ifdef RT_SPEC_FAMILY
template <class T> struct FamRec { T v; };
template <class T, int N>
__device__ __forceinline__ FamRec<T> fam_rec(const T (&ct)[N], const uint8_t* vary, const T* rt, int i) {
  constexpr int NW = (int)(sizeof(T) / 4);
  const uint32_t* cw = (const uint32_t*)(const void*)&ct[i];
  const __attribute__((address_space(4))) uint32_t* rw =
      (const __attribute__((address_space(4))) uint32_t*)(const void*)rt + (size_t)i * NW;
  uint32_t w[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) w[k] = vary[i * NW + k] ? rw[k] : cw[k];
  return FamRec<T>{__builtin_bit_cast(T, w)};
}
#define RT_REC(NAME, S, tab, TAB, I)                                                   \
  const auto NAME##_rec = fam_rec(rt_spec::TAB, rt_spec::VARY_##TAB, (S).tab, (I)); \
  const auto NAME = &NAME##_rec.v
#else
#define RT_REC(NAME, S, tab, TAB, I) const auto NAME = &(S).tab[I]
#endif

struct DS {                         // device view of RtDevScene
  cptr<RtObject> objects;
  cptr<RtTrav> trav;
  cptr<RtTrav> strav;               // shadow-ray walk of scenes without a transparent object
  cptr<RtTravC> trav_c;             // the same, compact (the generic walks with f32 culling)
  cptr<RtTravC> strav_c;
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
#ifndef RT_PLANE_SELF_SKIP
#define RT_PLANE_SELF_SKIP 1        // traversals: a plane distance provably below EPS skips its division
#endif
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

RT_FN bool leaf_inside(cptr<RtLeaf> L, V3 p, bool fin) {
  int k = L->kind;
  if (k == RT_N_PLANE) return false;                                        // :186-188
  V3 q = leaf_inv_xf(L, p, fin);
  if (k == RT_N_SPHERE) return len(sub(q, ld3(L->c))) <= L->r_eps;         // :70-74
  return q.x <= L->hi[0] && q.x >= L->lo[0] && q.y <= L->hi[1] &&          // :319-328
         q.y >= L->lo[1] && q.z <= L->hi[2] && q.z >= L->lo[2];
}

RT_FN bool leaf_on_surface(cptr<RtLeaf> L, V3 p, bool fin) {
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

RT_FN V3 leaf_normal(cptr<RtLeaf> L, V3 p, bool fin) {
  int k = L->kind;
  if (k == RT_N_PLANE) return ld3(L->pn[0]);                               // :182-184
  V3 q = leaf_inv_xf(L, p, fin);
  if (k == RT_N_SPHERE) {                                                  // :64-68
    V3 n = sub(q, ld3(L->c));
    return normalized(sub(xf(L->mat, n), ld3(L->mat_o)));
  }
  RT_SPEC_UNROLL
  for (int i = 0; i < 6; ++i)                                              // :292-317
    if (on_plane(L->pl[i], q)) return ld3(L->pn[i]);
  return {1.0, 1.0, 1.0};
}

// MathSphere::get_uv_coordinates (:82-114): the centre is subtracted BEFORE the inverse transform.
// tw, th > 0 (a textured object's texture size): the texel-boundary guard.  The texture lookup truncates
// x = u (tw - 1) and y = th - v (th - 1) - 1 (texture.rs:27-34), and u, v come from two acos and a sin that
// may differ from glibc's (the reference's libm) by an ulp (rt_acos, ocml's sin).  From those ulps the
// guard bounds how far the lane's x and y can be from glibc's (through sin's slope at phi, acos's slope
// 1 / sqrt(1 - r^2) at r, and every rounding on the way, times 16); a lane whose x or y lies within that
// bound of an integer (or of a clamp edge, or whose r is near +-1 or not finite) evaluates phi, sin(phi)
// and theta again with the correctly rounded rt_acos_cr / rt_sin_cr (rt_math.h) -- glibc's values except
// where glibc itself is not correctly rounded.  Far from a boundary both sides truncate to the same texel,
// and the guard costs ~30 flops per textured hit; a 4K frame has ~1e-12 of its hits near a boundary.
#ifndef RT_TEXEL_SAFE
#define RT_TEXEL_SAFE 1
#endif
// The rare lanes' recomputation.  The specialised programs inline it (their guard costs 0.4 %); the
// generic kernels call it: inlined at each of their shading sites, its double-double code made the
// generic 4K frame 3.6x slower (0.430 -> 1.554 ms, profiles/r09v_generic_ab.txt).
#ifdef RT_SPEC
#define RT_TEXEL_CR_FN __device__ __forceinline__
#else
#define RT_TEXEL_CR_FN __device__ __attribute__((noinline))
#endif
RT_TEXEL_CR_FN void sphere_uv_cr(double cy, double cz, bool flip, double* u, double* v) {
  double phi = rt_acos_cr(cy);                                             // rt_math.h
  if (isnan(phi)) phi = 0.0;
  double theta = rt_acos_cr(cz / rt_sin_cr(phi)) / (2.0 * PI_D);
  if (isnan(theta)) theta = 0.0;
  *v = phi / PI_D;
  *u = flip ? 1.0 - theta : theta;
}
__device__ __forceinline__ double ulp_bound(double a) { return fabs(a) * 0x1p-52 + 0x1p-1074; }
__device__ __forceinline__ bool near_int(double a, double m) { return !(fabs(a - rint(a)) > m); }   // NaN: near
RT_FN void sphere_uv(cptr<RtLeaf> L, V3 p, double* u, double* v, int tw = 0, int th = 0) {
  V3 q = xf(L->inv, sub(p, ld3(L->c)));           // per shaded hit only: no short form
  q = scale(normalized(q), 1.0 - EPS);
  const double cy = -((0.0 * q.x + 1.0 * q.y) + 0.0 * q.z);                  // up = (0,1,0)
  const double cz = (q.x * 0.0 + q.y * 0.0) + q.z * -1.0;                    // u_zero = (0,0,-1)
  const bool flip = (-1.0 * q.x + 0.0 * q.y) + 0.0 * q.z > 0.0;              // u_qrtr = (-1,0,0)
  double phi = rt_acos(cy);
  if (isnan(phi)) phi = 0.0;
  const double sp = sin(phi), r = cz / sp, ac = rt_acos(r);
  double theta = ac / (2.0 * PI_D);
  if (isnan(theta)) theta = 0.0;
  *v = phi / PI_D;
  *u = flip ? 1.0 - theta : theta;
  if (RT_TEXEL_SAFE && tw > 0) {
    const double x = *u * (double)(tw - 1), y = (double)th - (*v * (double)(th - 1)) - 1.0;
    const double ey = (double)(th - 1) * (2.0 * ulp_bound(phi) / PI_D + ulp_bound(*v)) + 2.0 * ulp_bound(y);
    const double er = 0x1p-50 + 4.0 * ulp_bound(phi) / fabs(sp);
    const double ea = fabs(r) * er / sqrt(fmax(1.0 - r * r, 0x1p-60)) + 2.0 * ulp_bound(ac);
    const double ex = (double)(tw - 1) * (ea / (2.0 * PI_D) + 2.0 * ulp_bound(*u)) + 2.0 * ulp_bound(x);
    if (!(fabs(r) < 1.0 - 0x1p-26) || near_int(x, 16.0 * ex) || near_int(y, 16.0 * ey))
      sphere_uv_cr(cy, cz, flip, u, v);                                      // the rare lanes
  }
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
      // |t| <= |num| / |v_d| (1 + 2^-52)^2 < EPS when |num| <= 2^-22 |v_d| (the product is exact or
      // rounds towards 0): never accepted.  A ray leaving the plane it starts on (the floor's shadow and
      // reflection rays) skips the division.
      if (POS && RT_PLANE_SELF_SKIP && fabs(num) <= 0x1p-22 * fabs(v_d)) return 0;
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
RT_FN bool leaf_filter(const DS& S, cptr<RtLeaf> L, V3 p) {
  const bool fin = wave_finite(p);
  const int nl = L->n_lit;
  if (nl >= 0) {                                   // conjunction of literals (rt_blob.h)
    RT_SPEC_UNROLL
    for (int k = 0; k < nl; ++k) {
      const int v = L->lit[k];
      RT_REC(LI, S, leaves, LEAVES, v >> 1);
      if (leaf_inside(LI, p, fin) != (bool)(v & 1)) return false;
    }
    return true;
  }
  uint32_t st = 0;
  const int e = L->prog_end;
  RT_SPEC_UNROLL
  for (int k = L->prog_begin; k < e; ++k) {
    const int op = S.prog[k].op, arg = S.prog[k].arg;
    if (op == RT_OP_INSIDE) {
      RT_REC(LI, S, leaves, LEAVES, arg);
      st = (st << 1) | (leaf_inside(LI, p, fin) ? 1u : 0u);
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

// The same test in f32 (RT_CULL_F32, the traversals of the megakernels and the deferred kernel): half
// the registers of the f64 culling ray, f32 instructions at twice the f64 issue rate, and the box
// bounds as 32-bit literals (VOP2 operands) in the specialised programs.  Conservative by construction:
//  * a ray is culled only if every origin coordinate is within RT_CULL32_COORD_MAX and its largest
//    direction component within [2^-10, 2^10] (cull_ray_f; otherwise every slab time is NaN, which
//    narrows nothing: min/max are IEEE minNum/maxNum);
//  * the f32 boxes are the f64 boxes grown by RT_CULL32_MARGIN = 4x the error of rounding such an origin
//    to f32, then rounded outward (scene.cpp f32_boxes), so the slab times computed from the rounded
//    origin bound those of the exact origin against a box that still contains the f64 box;
//  * what remains is relative: fl32(box - o) * rcp32(fl32(d)) is within 2^-21 of its exact value, and
//    the comparison tn <= tf allows 2^-18 of slack on each side;
//  * a direction component below 2^-100 is taken as zero (inv = +-inf): reaching a slab RT_CULL32_MARGIN
//    away would take t > 2^93, where the largest component (>= 2^-10) has left every box (|bounds| <= 1e6);
//    (box - o) * inf is +-inf, or NaN (narrows nothing) when box - o == 0;
//  * the only infinite time that reaches the comparison is tn = +inf from such a zero component with
//    the origin outside its slab (the ray never enters it: exact), and tf is finite (some component
//    is >= 2^-10), so the slack never hides an infinity.
// RT_CULL_FMA (a diagnostic variant, below): a slab time is one fma, fma(box, inv, -fl32(o * inv)) =
// (box - o - o e1) inv (1 + e2), |e1|, |e2| <= 2^-24: the exact time of a ray from an origin moved by
// |o e1| <= 2^16 * 2^-24 = 2^-8 on top of the f32 rounding (<= 2^-9), together under the margin, the
// rest relative as above.  A component below 2^-100 then takes inv = +-2^100 (a direction of magnitude
// 2^-100: over any t at which the ray can be in a finite box, t < 2^31 since every finite box and the
// origin lie within 1e6 in EVERY axis (scene.cpp box_infinite), that moves the ray by < 2^-69), not
// +-inf: fma(lo, inf, -o * inf) is NaN for the bound on one side of the origin and +-inf for the other,
// and minNum(NaN, +inf) made +inf the near time of a ray parallel to a slab it starts inside
// (tests/test_gpu_cull_edges.py found it: a shadow ray with d.x == 0 toward a light at the same x,
// profiles/r09u_culldiff.txt).
// The specialised programs take it (4K globes 0.3184 -> 0.2868 ms); the generic kernels keep the f64
// test: with f32 tests the generic walks of fractal.scene (171 objects, ray trees) ran the same
// instructions and wave-cycles in 2.9x the time (its wavefront level-0 trace 0.59 -> 1.69 ms per
// frame, profiles/r09p_*), and the generic 4K frame gained nothing (0.463 vs 0.457-0.487 ms).
#ifndef RT_CULL_F32
#ifdef RT_SPEC
#define RT_CULL_F32 1
#else
#define RT_CULL_F32 0
#endif
#endif
// RT_CULL_FMA: each slab time as one fma (above) -- v_fmamk_f32 with the bound as its literal, one
// instruction where (box - o) * inv takes two.  Conservative, and the
// 4K kernel's VALU instructions per wave fell 1 174.6 -> 1 141.8, but every config ran slower (4K 0.2732
// -> 0.2737 ms, sphere 0.0146 -> 0.0147, 1080p d5 0.0816 -> 0.0830; profiles/r09r_fma_slab_ab.txt):
// kept as a diagnostic variant, off.
#ifndef RT_CULL_FMA
#define RT_CULL_FMA 0
#endif
#if RT_CULL_FMA
struct CullRayF { float ix, iy, iz, nx, ny, nz; };   // 1 / d and -o / d (f32)
#else
struct CullRayF { float ix, iy, iz, ox, oy, oz; };
#endif
__device__ __forceinline__ float cull_rcp_f(float x) {
  return fabsf(x) < 0x1p-100f ? copysignf(RT_CULL_FMA ? 0x1p100f : __builtin_inff(), x) : __builtin_amdgcn_rcpf(x);
}
__device__ __forceinline__ CullRayF cull_ray_f(V3 o, V3 d) {
  const double ad = fmax(fmax(fabs(d.x), fabs(d.y)), fabs(d.z));
  const bool ok = fabs(o.x) <= RT_CULL32_COORD_MAX && fabs(o.y) <= RT_CULL32_COORD_MAX &&
                  fabs(o.z) <= RT_CULL32_COORD_MAX && ad >= 0x1p-10 && ad <= 0x1p10;
  const float nan = __builtin_nanf("");
  const float ix = ok ? cull_rcp_f((float)d.x) : nan, iy = ok ? cull_rcp_f((float)d.y) : nan,
              iz = ok ? cull_rcp_f((float)d.z) : nan;
#if RT_CULL_FMA
  return {ix, iy, iz, -((float)o.x * ix), -((float)o.y * iy), -((float)o.z * iz)};
#else
  return {ix, iy, iz, (float)o.x, (float)o.y, (float)o.z};
#endif
}
template <class P> __device__ __forceinline__ bool fbox_may_hit(P lo, P hi, const CullRayF& r, float tmax) {
#if RT_CULL_FMA
  const float ax = __builtin_fmaf(lo[0], r.ix, r.nx), bx = __builtin_fmaf(hi[0], r.ix, r.nx);
  const float ay = __builtin_fmaf(lo[1], r.iy, r.ny), by = __builtin_fmaf(hi[1], r.iy, r.ny);
  const float az = __builtin_fmaf(lo[2], r.iz, r.nz), bz = __builtin_fmaf(hi[2], r.iz, r.nz);
#else
  const float ax = (lo[0] - r.ox) * r.ix, bx = (hi[0] - r.ox) * r.ix;
  const float ay = (lo[1] - r.oy) * r.iy, by = (hi[1] - r.oy) * r.iy;
  const float az = (lo[2] - r.oz) * r.iz, bz = (hi[2] - r.oz) * r.iz;
#endif
  const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
  const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
  return tn * (1.0f - 0x1p-18f) <= __builtin_fmaf(fabsf(tf), 0x1p-18f, tf);
}
__device__ __forceinline__ float cull_tmax_f(double t) { return (float)cull_tmax(t); }
#if RT_CULL_F32
// The traversals' culling ray and tests, f32 (above) or f64 (box_may_hit)
typedef CullRayF CullR;
typedef float CullT;
#define RT_CULL_RAY(o, d) cull_ray_f(o, d)
#define RT_CULL_TMAX(t) cull_tmax_f(t)
#define RT_BOX_MAY_HIT(R, lo, hi, cr, tm) fbox_may_hit((R)->f##lo, (R)->f##hi, cr, tm)
#else
typedef CullRay CullR;
typedef double CullT;
#define RT_CULL_RAY(o, d) cull_ray(o, d)
#define RT_CULL_TMAX(t) cull_tmax(t)
#define RT_BOX_MAY_HIT(R, lo, hi, cr, tm) box_may_hit((R)->lo, (R)->hi, cr, tm)
#endif
// Hierarchy node accessors: the walks' lambdas take a node of either form -- RtTrav (the specialised
// programs' constexpr tables, and f64-culling builds) or RtTravC (the generic walks with f32 culling).
__device__ __forceinline__ int node_obj(cptr<RtTrav> T) { return T->obj; }
__device__ __forceinline__ int node_skip(cptr<RtTrav> T) { return T->skip; }
__device__ __forceinline__ int node_cull(cptr<RtTrav> T) { return T->cull; }
__device__ __forceinline__ int node_shadow_skip(cptr<RtTrav> T) { return T->shadow_skip; }
template <class CR, class TM> __device__ __forceinline__ bool node_may_hit(cptr<RtTrav> T, const CR& cr, TM tm) {
  return RT_BOX_MAY_HIT(T, blo, bhi, cr, tm);
}
__device__ __forceinline__ int node_obj(cptr<RtTravC> T) { return T->obj; }
__device__ __forceinline__ int node_skip(cptr<RtTravC> T) { return (int)(T->skip_flags & 0x0fffffffu); }
__device__ __forceinline__ int node_cull(cptr<RtTravC> T) { return (int)((T->skip_flags >> 28) & 3u); }
__device__ __forceinline__ int node_shadow_skip(cptr<RtTravC> T) { return (int)(T->skip_flags >> 30); }
__device__ __forceinline__ bool node_may_hit(cptr<RtTravC> T, const CullRayF& cr, float tm) {
  return fbox_may_hit(T->lo, T->hi, cr, tm);
}

// The range the host proves constant hit filters for (RtLeaf::filter_const): cull_ray's valid range
// (origin within 1e6, largest direction component within [1e-100, 1e100]).
__device__ __forceinline__ bool const_filter_range(V3 o, V3 d) {
  const double ad = fmax(fmax(fabs(d.x), fabs(d.y)), fabs(d.z));
  return fabs(o.x) <= RT_CULL_COORD_MAX && fabs(o.y) <= RT_CULL_COORD_MAX && fabs(o.z) <= RT_CULL_COORD_MAX &&
         ad >= 1e-100 && ad <= 1e100;
}

// The object's oriented box (RtObject::obb_leaf, scene.cpp obb): may the segment t in [0, tmax]
// meet the leaf-frame box olo/ohi?  The ray is taken to the leaf's frame with the leaves' own
// arithmetic; outside the range the host's margins are proven for (|o| <= 1e6, unit-length
// directions) the answer is yes.  The refraction kernels (SHARE: 4 waves/SIMD at 115-119 VGPRs)
// do not take it: the test's code alone made spinning_globes (no oriented box) 2.7 % slower
// (profiles/r02cg_obb_ab.txt).
#ifndef RT_OBB
#define RT_OBB 1
#endif
__device__ __forceinline__ bool obb_may_hit(const DS& S, cptr<RtObject> O, V3 ro, V3 rd, CullT tmax) {
  RT_REC(R, S, leaves, LEAVES, O->obb_leaf);
  const double ad = fmax(fmax(fabs(rd.x), fabs(rd.y)), fabs(rd.z));
  if (!(ad >= 0.25 && ad <= 4.0 && fabs(ro.x) <= 1e6 && fabs(ro.y) <= 1e6 && fabs(ro.z) <= 1e6)) return true;
  const V3 o = xf(R->inv, ro);
  const V3 d = sub(xf(R->inv, rd), ld3(R->inv_o));
  return RT_BOX_MAY_HIT(O, olo, ohi, RT_CULL_RAY(o, d), tmax);   // leaf-frame ray: cull_ray*'s own range checks
}

// ------------------------------------------------------------------ traversal (raytracer.rs)
// Both traversals walk the object hierarchy (RtTrav, pre-order over contiguous draw-order runs)
// wave-coherently: `i` is uniform, a lane that misses a group resumes at its skip index, and the
// wave jumps over a group no lane entered.  walk_trav calls group(T) for a group node (does this
// lane enter it?) and object(T) for an object node the lane reaches.
// RT_SPEC (the scene-specialised kernel, k_spec.hip): the hierarchy is a constexpr table, so the
// walk is unrolled at compile time into nested branches -- every node's fields, every object's and
// leaf's record are constants, and a branch no lane takes is jumped over by the hardware (EXEC = 0),
// exactly the generic walk's skip.
#ifdef RT_SPEC
#define RT_INL __attribute__((always_inline))
template <int N> struct IC { static constexpr int value = N; };
template <int I, int END, class F>
__device__ __forceinline__ void spec_for(F&& f) {
  if constexpr (I < END) {
    f(IC<I>{});
    spec_for<I + 1, END>(f);
  }
}
// (RT_SPEC_FAMILY: a node's obj and skip are shared by every member of the family, spec.hip checks)
template <bool SORD, int I, int END, class G, class O>
__device__ __forceinline__ void spec_walk(const DS& S, G& group, O& object) {
  if constexpr (I < END) {
    constexpr RtTrav T = SORD ? rt_spec::STRAV[I] : rt_spec::TRAV[I];
    auto body = [&](cptr<RtTrav> TP) RT_INL {
      if constexpr (T.obj < 0) {
        if (group(TP)) spec_walk<SORD, I + 1, T.skip>(S, group, object);
        spec_walk<SORD, T.skip, END>(S, group, object);
      } else {
        object(TP);
        spec_walk<SORD, I + 1, END>(S, group, object);
      }
    };
    if constexpr (SORD) {
      RT_REC(TP, S, strav, STRAV, I);
      body(TP);
    } else {
      RT_REC(TP, S, trav, TRAV, I);
      body(TP);
    }
  }
}
#else
#define RT_INL
#endif
// STOP (the shadow walk's early-out): stop(T) after an object node says whether this lane is done;
// once no lane walks on, the generic walk ends (the spec walk's remaining branches are skipped by
// the hardware, EXEC = 0).
template <bool SORD, bool STOP = false, class G, class O>
__device__ __forceinline__ void walk_trav(const DS& S, G&& group, O&& object, bool* done = nullptr) {
#ifdef RT_SPEC
  spec_walk<SORD, 0, SORD ? rt_spec::N_STRAV : rt_spec::N_TRAV>(S, group, object);
#else
  // f32 culling: the compact nodes (RtTravC: two per scalar-cache line)
#ifndef RT_TRAV_COMPACT
#define RT_TRAV_COMPACT 1
#endif
#if RT_CULL_F32 && RT_TRAV_COMPACT
  const cptr<RtTravC> TR = SORD ? S.strav_c : S.trav_c;
#else
  const cptr<RtTrav> TR = SORD ? S.strav : S.trav;
#endif
  const int n_tr = SORD ? S.n_strav : S.n_trav;
  int resume = 0;
  for (int i = 0; i < n_tr;) {
    const auto T = &TR[i];
    const bool act = i >= resume;
    if (node_obj(T) < 0) {                               // group node
      const bool in = act && group(T);
      if (act && !in) resume = node_skip(T);
      i = __ballot(in) ? i + 1 : node_skip(T);
      continue;
    }
    ++i;
    if (act) object(T);
    if constexpr (STOP)
      if (__ballot(!*done) == 0) break;
  }
#endif
}

// Nearest hit over all objects in draw order: accept d if d > EPS && d < nearest
// (raytracer.rs:141-150).  The acceptance test is pure, so it runs BEFORE the (pure) CSG
// filter: candidates that cannot win never pay for the sibling is_inside tests.
// SHARE: concentric sphere leaves reuse their ray terms (SphereShare); it keeps three doubles live
// across the leaf loop, so only kernels with register headroom take it (see trace()).
template <bool SHARE = false, bool OBB = !SHARE>
RT_FN int nearest_hit(const DS& S, V3 ro, V3 rd, double* dist) {
  double best = INFINITY;
  int bobj = -1;
  SphereShare shr = {0.0, 0.0, 0.0};
  const CullR cr = RT_CULL_RAY(ro, rd);
  const bool cf_ok = SHARE && RT_CONST_FILTER && const_filter_range(ro, rd);
  const bool fin = wave_finite(ro, rd);
  // NORDER (reflection-only kernels): the objects in S.strav's order, largest regions first, so an
  // early hit on a big object culls what lies behind it.  Exact: a candidate equal to the best
  // distance so far wins when its object comes earlier in DRAW order (o < bobj), which is the
  // reference's first-visited-wins rule (raytracer.rs:141-150) for any visiting order.
  constexpr bool NORDER = RT_NEAREST_ORDER && OBB;
  auto group = [&](auto T) RT_INL { return node_may_hit(T, cr, RT_CULL_TMAX(best)); };
  auto object = [&](auto T) RT_INL {
    // the object's cull kind and box come from the node's copy (RtTrav): one scalar load for the
    // node decides the common case; the object's own record is read only once its box passes
    if (node_cull(T) == RT_CULL_ALWAYS) return;
    if (node_cull(T) == RT_CULL_BOX && !node_may_hit(T, cr, RT_CULL_TMAX(best))) return;
    const int o = node_obj(T);
    RT_REC(O, S, objects, OBJECTS, o);
    if (RT_OBB && OBB && O->obb_leaf >= 0 && !obb_may_hit(S, O, ro, rd, RT_CULL_TMAX(best))) return;
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    RT_SPEC_UNROLL
    for (int l = lb; l < le; ++l) {
      RT_REC(L, S, leaves, LEAVES, l);
      if (O->leaf_cull) {
        if (L->cull == RT_CULL_ALWAYS) continue;
        if (L->cull == RT_CULL_BOX && !RT_BOX_MAY_HIT(L, blo, bhi, cr, RT_CULL_TMAX(best))) continue;
      }
      double t0 = 0.0, t1 = 0.0;
      int n = leaf_candidates<true>(L, ro, rd, fin, &t0, &t1, SHARE ? &shr : nullptr);
      const bool filtered = L->prog_end != L->prog_begin && !(cf_ok && L->filter_const);
      if (n >= 1 && t0 > EPS && (t0 < best || (NORDER && t0 == best && o < bobj)) &&
          (!filtered || leaf_filter(S, L, add(ro, scale(rd, t0))))) {
        best = t0; bobj = o;
      }
      if (n >= 2 && t1 > EPS && (t1 < best || (NORDER && t1 == best && o < bobj)) &&
          (!filtered || leaf_filter(S, L, add(ro, scale(rd, t1))))) {
        best = t1; bobj = o;
      }
    }
  };
  walk_trav<NORDER>(S, group, object);
  *dist = best;
  return bobj;
}

// Product of the transparencies of every filtered hit with EPS < d < dist (raytracer.rs:181-197).
// Early-out once the product is exactly 0 (it stays 0: every factor is finite, checked on the
// host), objects of transparency exactly 1.0 are skipped (x * 1.0 == x).
// SORDER (reflection-only kernels): walk S.strav, the likeliest occluders first (scene.cpp
// shadow_order) -- every transparency is +-0 there, so the first filtered hit decides and the
// order is free.  The early return ends the walk: `done` skips the rest of it (in the generic
// walk a finished lane only rides along; the wave leaves once every lane is done).
template <bool SHARE = false, bool OBB = !SHARE, bool SORDER = OBB>
RT_FN double shadow_transparency(const DS& S, V3 p, V3 dir, double dist) {
  RT_OPAQUE(p.x);
  RT_OPAQUE(p.y);
  RT_OPAQUE(p.z);
  double tr = 1.0;
  bool done = false;
  SphereShare shr = {0.0, 0.0, 0.0};
  const CullR cr = RT_CULL_RAY(p, dir);
  const bool cf_ok = SHARE && RT_CONST_FILTER && const_filter_range(p, dir);
  const bool fin = wave_finite(p, dir);
  const CullT tmax = RT_CULL_TMAX(dist);
  auto group = [&](auto T) RT_INL { return !done && node_may_hit(T, cr, tmax); };
  auto object = [&](auto T) RT_INL {
    if (done) return;
    if (node_shadow_skip(T) || node_cull(T) == RT_CULL_ALWAYS) return;   // the node's copies (see nearest_hit)
    if (node_cull(T) == RT_CULL_BOX && !node_may_hit(T, cr, tmax)) return;
    RT_REC(O, S, objects, OBJECTS, node_obj(T));
    if (RT_OBB && OBB && O->obb_leaf >= 0 && !obb_may_hit(S, O, p, dir, tmax)) return;
    const double tobj = O->transparency;
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    RT_SPEC_UNROLL
    for (int l = lb; l < le; ++l) {
      RT_REC(L, S, leaves, LEAVES, l);
      if (O->leaf_cull) {
        if (L->cull == RT_CULL_ALWAYS) continue;
        if (L->cull == RT_CULL_BOX && !RT_BOX_MAY_HIT(L, blo, bhi, cr, tmax)) continue;
      }
      double t0 = 0.0, t1 = 0.0;
      int n = leaf_candidates<true>(L, p, dir, fin, &t0, &t1, SHARE ? &shr : nullptr);
      const bool filtered = L->prog_end != L->prog_begin && !(cf_ok && L->filter_const);
      if (n >= 1 && t0 > EPS && t0 < dist && (!filtered || leaf_filter(S, L, add(p, scale(dir, t0))))) {
        tr *= tobj;
        if (tr == 0.0 && S.shadow_early_out) { done = true; return; }
      }
      if (n >= 2 && t1 > EPS && t1 < dist && (!filtered || leaf_filter(S, L, add(p, scale(dir, t1))))) {
        tr *= tobj;
        if (tr == 0.0 && S.shadow_early_out) { done = true; return; }
      }
    }
  };
  walk_trav<RT_SHADOW_ORDER && SORDER, true>(S, group, object, &done);
  return done ? 0.0 : tr;
}

// Normal and UV of top-level object O at point p: RTObject shape get_normal / get_uv_coordinates,
// with CSG's is_on_surface / is_inside evaluated bottom-up over the post-order node list
// (csg.rs:98-168) and the descent a-then-b of csg.rs:104-121 / :161-167.
RT_FN void object_normal_uv(const DS& S, cptr<RtObject> O, V3 p, bool want_uv, V3* n,
                                 double* u, double* v) {
  cptr<RtNode> N = S.nodes + O->node_begin;
  const int cnt = O->node_count;
  const bool fin = wave_finite(p);
  *u = 0.0;
  *v = 0.0;
  // want_uv: the object is textured; its texture's size arms sphere_uv's texel-boundary guard
  const int tw = want_uv ? S.textures[O->tex].w : 0, th = want_uv ? S.textures[O->tex].h : 0;
  if (cnt == 1) {
    RT_REC(L, S, leaves, LEAVES, N[0].leaf);
    *n = leaf_normal(L, p, fin);
    if (want_uv && L->kind == RT_N_SPHERE) sphere_uv(L, p, u, v, tw, th);
    return;
  }
  uint32_t in = 0, on = 0;
  RT_SPEC_UNROLL
  for (int i = 0; i < cnt; ++i) {
    const int nk = N[i].kind, na = N[i].a, nb = N[i].b, nl = N[i].leaf;
    bool bi, bo;
    if (nk < RT_N_UNION) {
      RT_REC(L, S, leaves, LEAVES, nl);
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
  RT_SPEC_UNROLL
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
  RT_SPEC_UNROLL
  for (int l = lb; l < le; ++l) {
    if (!((__ballot(sel == l) >> lane) & 1)) continue;
    RT_REC(L, S, leaves, LEAVES, l);
    *n = leaf_normal(L, p, fin);
    if (want_uv && L->kind == RT_N_SPHERE) sphere_uv(L, p, u, v, tw, th);
  }
  if (neg) *n = scale(*n, -1.0);
}

// PixmapTexture::get_color_at (texture.rs:27-34) on RGBA8 texels, /255.0 (sceneparser/texture.rs:29-33)
RT_FN Col texture_color(const DS& S, int tex, double u, double v) {
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
// inside_test's "outside" answer without the square root and the division, for cin = d / (len(a) * nl)
// with q = dot(a, a) (len(a) = sqrt(q)): when d > 0 and d^2 > 1e-30 q nl^2 (1 + 2^-40), with the right
// side a normal double, the computed cin exceeds 1e-15 -- sqrt, product and quotient round by 2^-53
// each, the squares and products here by as much, and 2^-40 covers them all -- so inside_test answers
// false.  Anything else (NaN, overflow, grazing, inside) takes the exact path.  A wave of hits seen
// from outside (floor pixels, every primary hit) skips len() and the division.
#ifndef RT_INSIDE_FAST
#define RT_INSIDE_FAST 1
#endif
__device__ __forceinline__ bool outside_certain(double d, double q, double nl) {
  const double rhs = (1e-30 * q) * (nl * nl) * (1.0 + 0x1p-40);
  return d > 0.0 && rhs >= 0x1p-1000 && d * d > rhs;
}

// ang / (PI / 2) of the Lambert term (raytracer.rs:216-218) for ang in [0, PI/2): an acos result there is
// +0 or at least acos(1 - 2^-53) > 1e-8 (never subnormal), so div_core's conditions hold (no scaling in
// either v_div_scale; a zero numerator keeps its sign through v_div_fixup): the compiler's division
// minus its identities, bit-identical.
__device__ __forceinline__ double lambert_ratio(double ang) {
#if RT_FAST_SQRT
  return div_core(ang, PI_D / 2.0);
#else
  return ang / (PI_D / 2.0);
#endif
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
// nlen (optional): len(normal) of the normalised normal, the denominator term the Lambert angles and the
// inside test take (vector.rs:57-59) -- formed once here.  Objects whose normal is a constant (a plane:
// RtObject::unit_normal) take the host's normalised normal and its length (the same IEEE operations on the
// same values: bit-identical), so a wave of floor hits skips the normalisation and the length.
#ifndef RT_UNIT_NORMAL
#define RT_UNIT_NORMAL 1
#endif
__device__ __forceinline__ void shade_inputs(const DS& S, int oi, V3 p, V3* nrm, Col* c, double* transp,
                                             double* refl, double* nlen = nullptr) {
  RT_OPAQUE(p.x);                          // RT_SPEC: keep the per-object work on p in the light loop
  RT_OPAQUE(p.y);                          // (see RT_OPAQUE)
  RT_OPAQUE(p.z);
  bool unit = false;
  auto shade = [&](cptr<RtObject> O) RT_INL {
    double u = 0.0, v = 0.0;                 // a plane's UV is Err -> (0, 0) (math_shapes.rs:196-198)
    if (RT_UNIT_NORMAL && nlen && O->unit_normal) {
      *nrm = ld3(O->nunit);
      *nlen = O->nunit_len;
      unit = true;
    } else {
      object_normal_uv(S, O, p, O->textured != 0, nrm, &u, &v);
    }
    *c = O->textured ? texture_color(S, O->tex, u, v) : Col{O->color[0], O->color[1], O->color[2]};
    *transp = O->transparency;
    *refl = O->reflectivity;
  };
#ifdef RT_SPEC
  // every object's inputs are constants: one branch per object, taken by the lanes that hit it
  spec_for<0, rt_spec::N_OBJECTS>([&](auto I) RT_INL {
    constexpr int o = decltype(I)::value;
    if (oi == o) {
      RT_REC(O, S, objects, OBJECTS, o);
      shade(O);
    }
  });
#else
  uint64_t todo = __ballot(oi >= 0);
  while (todo) {
    const int o = __builtin_amdgcn_readlane(oi, (int)__builtin_ctzll(todo));
    const uint64_t mine = __ballot(oi == o);
    todo &= ~mine;
    // test membership through the ballot mask, not `oi == o`: an equality lets the optimiser
    // substitute the per-lane oi for the uniform o and the loads below turn into VMEM again.
    if ((mine >> __lane_id()) & 1) shade(&S.objects[o]);
  }
#endif
  if (!unit) {
    *nrm = normalized(*nrm);
    if (nlen) *nlen = len(*nrm);
  }
}

template <class A, class B> struct same_type { static constexpr bool value = false; };
template <class A> struct same_type<A, A> { static constexpr bool value = true; };


// Ray-debugger recording (raytracer.rs:17-19, :155-157, :282-284; ray_debugger.rs:92-137).
// NoRec compiles to nothing in the render kernels; RtRayRecord slots are written in ray START
// order and `order` lists them in the reference's callback order (a ray reports after its
// children: post-order).
struct NoRec {
  __device__ __forceinline__ int begin(int, int, V3, V3, double, int, V3) { return 0; }
  __device__ __forceinline__ void finish(int, Col) {}
};
#ifndef __HIPCC_RTC__
using RtRayRecord = rt_ray_record;
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
#endif

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
#define RT_LDS_FRAMES_CHAIN 0          // round 6: every chain frame in the wave's pool (rows_pool_slots)
#endif
// Refraction frames also carry the pending reflection ray (P, D, rp: 7 doubles); the first
// KLR of them go to LDS after the KL colour frames, [frame][component][lane] likewise.
#ifndef RT_LDS_RFRAMES
#define RT_LDS_RFRAMES 1
#endif

// The wave's frame POOL (KP > 0, chain and reflection-only kernels, round 5): instead of KL frames per
// lane, the wave's LDS holds KP frame slots shared by its 64 lanes.  In those modes every hit spawns at
// most one ray, so the lanes still walking push their frame f in the same iteration f: one ballot gives
// the pushing lanes m, each takes slot start + (its rank in m) (mbcnt), and (m, start) are kept per f
// (pool_mask / pool_start) so that a lane folding its frame f later finds its slot again.  Lanes whose
// chains are short leave their share to the long ones: a spinning_globes wave needs ~2 frames per lane
// on average but up to 10 for some lanes, so the fixed per-lane layout either spilled the deep frames
// to scratch (KL = 5: 48.7 MB of HBM per 1080p frame) or cost occupancy.  Slots past KP, and frames of
// pixels whose chain outgrows the pool, use the private array (scratch).  The first KL frames of every
// lane keep their fixed per-lane LDS slots (most chains are that short, and a fixed slot costs no
// ballot, no rank and no header reads); the pool serves the deeper ones.  Layout at the wave's base lp:
// [KL][4][64] per-lane frames, [RT_MAX_DEPTH_CAP] u64 masks, [RT_MAX_DEPTH_CAP] u32 starts, then [4][KP]
// doubles (component-major: the lanes of one push write consecutive doubles).
constexpr int RT_POOL_HDR = RT_MAX_DEPTH_CAP + RT_MAX_DEPTH_CAP / 2;      // header doubles
#define LDS_U64 __attribute__((address_space(3))) uint64_t
#define LDS_U32 __attribute__((address_space(3))) uint32_t
#define LDS_U8 __attribute__((address_space(3))) uint8_t
// Pool slots hold (A, hit object) instead of (A, w) (round 6).  Outside the ray-tree mode a frame's
// weight is a function of the hit object alone: a refraction frame's w is the object's transparency; a
// reflection frame's is rp = TIR ? refl + (1 - refl) * transp : refl (raytracer.rs:261-265), and a TIR
// hit refracts only where transp != 0, which in these modes forces refl == +-0, so rp = 0 + 1 * transp
// = transp exactly; without TIR a reflecting object has transp == 0 (else it would have refracted), so
// w = refl.  Hence w = (transp != 0 ? transp : refl) of the frame's object (frame_weight), bit for bit,
// and a slot is 3 doubles + 1 byte: 25 B instead of 32.  Scenes of more than 256 objects keep w.
#ifndef RT_POOL_OBJ_INDEX
#define RT_POOL_OBJ_INDEX 1
#endif
template <int KP, bool PIDX> constexpr int pool_doubles() { return PIDX ? 3 * KP + (KP + 7) / 8 : 4 * KP; }
// the weight of a frame whose hit object is o (see RT_POOL_OBJ_INDEX)
__device__ __forceinline__ double frame_weight(const DS& S, int o) {
#ifdef RT_SPEC
  double w = 0.0;
  spec_for<0, rt_spec::N_OBJECTS>([&](auto I) RT_INL {
    constexpr int k = decltype(I)::value;
    RT_REC(O, S, objects, OBJECTS, k);
    const double t = O->transparency;
    if (o == k) w = t != 0.0 ? t : O->reflectivity;
  });
  return w;
#else
  const double t = S.objects[o].transparency;          // per-lane loads (the generic kernels)
  return t != 0.0 ? t : S.objects[o].reflectivity;
#endif
}
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {                 // set lanes of m below this one
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// get_ray_color (raytracer.rs:132-287) for one primary ray, recursion unrolled onto a per-lane
// frame stack.  REFR = the scene has a transparent object (refraction frames need more state).
// KL > 0: frames 0..KL-1 of the stack are in LDS at lf[(f * 4 + c) * 64] (lf = this lane's slot);
// KLR > 0 (REFR): the pending-reflection state of frames 0..KLR-1 at lf[(KL * 4 + f * 7 + c) * 64].
// KP > 0 (not TREE, no recorder): frames KL.. go to the wave's pool of KP slots (above), after the KL
// per-lane frames at lp.
// CHAIN (REFR scenes with RtDevScene::ray_chains): every hit spawns at most one ray, so a refraction
// frame never carries a pending reflection: frames are (A, w) as in the reflection-only kernels.
template <bool REFR, class Rec = NoRec, int KL = 0, bool FC = false, int KLR = 0, bool CHAIN = false, int KP = 0>
RT_FN Col trace(const DS& S, V3 ro, V3 rd, int max_depth, Rec* rec = nullptr, lds_f64* lf = nullptr,
                lds_f64* lp = nullptr) {
  double fA[RT_MAX_DEPTH_CAP][3];     // parent colour already intensified by (1 - w)
  double fW[RT_MAX_DEPTH_CAP];        // child weight w (transparency or reflectivity)
  constexpr bool POOL = KP > 0 && !(REFR && !CHAIN) && same_type<Rec, NoRec>::value;
  // pool slots hold the hit object instead of w (RT_POOL_OBJ_INDEX); the scene has <= 256 objects (host)
  constexpr bool PIDX = POOL && RT_POOL_OBJ_INDEX;
  // frames 0..KL-1 stay in the lanes' own LDS slots (lf); the pool serves frames KL.. (after them at lp)
  LDS_U64* const pool_mask = (LDS_U64*)(lp + KL * 4 * 64);
  LDS_U32* const pool_start = (LDS_U32*)(lp + KL * 4 * 64 + RT_MAX_DEPTH_CAP);
  lds_f64* const pool = lp + KL * 4 * 64 + RT_POOL_HDR;
  LDS_U8* const pool_obj = (LDS_U8*)(pool + 3 * KP);             // PIDX: [KP] object bytes after [3][KP] doubles
  uint32_t pool_used = 0;             // wave-uniform: slots taken by the pushes so far
  auto put_frame = [&](int f, Col A, double w) {
    if (KL > 0 && f < KL) {
      lf[(f * 4 + 0) * 64] = A.r; lf[(f * 4 + 1) * 64] = A.g; lf[(f * 4 + 2) * 64] = A.b; lf[(f * 4 + 3) * 64] = w;
    } else {
      fA[f][0] = A.r; fA[f][1] = A.g; fA[f][2] = A.b; fW[f] = w;
    }
  };
  auto get_frame = [&](int f, Col* A, double* w) {
    if (POOL && f >= KL) {
      const uint32_t slot = pool_start[f] + lane_rank(pool_mask[f]);
      if (slot < (uint32_t)KP) {
        *A = {pool[slot], pool[KP + slot], pool[2 * KP + slot]};
        if constexpr (PIDX) *w = frame_weight(S, pool_obj[slot]);
        else *w = pool[3 * KP + slot];
        return;
      }
    }
    if (KL > 0 && f < KL) {
      *A = {lf[(f * 4 + 0) * 64], lf[(f * 4 + 1) * 64], lf[(f * 4 + 2) * 64]}; *w = lf[(f * 4 + 3) * 64];
    } else {
      *A = {fA[f][0], fA[f][1], fA[f][2]}; *w = fW[f];
    }
  };
  // POOL: the frame every lane still walking pushes in this iteration (they are all at frame f)
  auto pool_push = [&](bool push, int f, Col A, double w, int obj) {
    const uint64_t m = __ballot(push);
    const uint32_t start = pool_used;
    if (push) {
      const uint32_t slot = start + lane_rank(m);
      if (slot < (uint32_t)KP) {
        pool[slot] = A.r; pool[KP + slot] = A.g; pool[2 * KP + slot] = A.b;
        if constexpr (PIDX) pool_obj[slot] = (uint8_t)obj;
        else pool[3 * KP + slot] = w;
      } else {
        fA[f][0] = A.r; fA[f][1] = A.g; fA[f][2] = A.b; fW[f] = w;
      }
      pool_mask[f] = m;                 // every pushing lane writes the same (m, start)
      pool_start[f] = start;
    }
    pool_used = start + (uint32_t)__builtin_popcountll(m);
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
  constexpr bool RECORD = !same_type<Rec, NoRec>::value;
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
  for (int iter = 0;; ++iter) {
    bool descend = false;
    [[maybe_unused]] bool pushing = false;        // POOL: this lane pushes frame `iter` (its sp) now
    [[maybe_unused]] Col push_A = {0.0, 0.0, 0.0};
    [[maybe_unused]] double push_w = 0.0;
    double t_hit;
    int oi;
    oi = nearest_hit<SHARE, OBB>(S, ro, rd, &t_hit);
    const V3 p = add(ro, scale(rd, t_hit));                               // :162
    if constexpr (RECORD) slot = rec->begin(depth, ray_type, ro, rd, t_hit, oi, p);
    V3 nrm = {0.0, 0.0, 0.0};
    Col c = {0.0, 0.0, 0.0}, L = {0.0, 0.0, 0.0};
    double transp = 0.0, refl = 0.0, nlen = 0.0;
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
        RT_REC(lt, S, lights, LIGHTS, k);
        const V3 lv = sub(ld3(lt->p), p);
        double ll, ill;
        len_inv(lv, &ll, &ill);
        const V3 sdir = scale(lv, ill);                                    // normalized(lv)
        double t;                                                          // :176-197
        t = shadow_transparency<SHARE, OBB>(S, p, sdir, ll);
        if (!have_shading) {
          shade_inputs(S, oi, p, &nrm, &c, &transp, &refl, &nlen);
          L = cmul<FC>(c, in_range<FC>(0.6, 0.6, 0.6));                      // ambient (:172)
          have_shading = true;
        }
        if (t == 0.0) continue;                                            // :199-227
        double ang = rt_acos(dot(sdir, nrm) / (len(sdir) * nlen));
        if (ang >= PI_D / 2.0) ang = PI_D - ang;
        const double inten = (ang < (PI_D / 2.0) && ang >= 0.0) ? 1.0 - lambert_ratio(ang) : 0.0;
        const Col lc = intensify<FC>(intensify<FC>(Col{lt->col[0], lt->col[1], lt->col[2]}, inten), t);
        L = cadd<FC>(L, cmul<FC>(c, lc));
      }
      if (!have_shading) {
        shade_inputs(S, oi, p, &nrm, &c, &transp, &refl, &nlen);
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
        const double d = dot(nd, nrm);
        if (!(RT_INSIDE_FAST && outside_certain(d, dot(nd, nd), nlen)))
          inside = inside_test(d / (len(nd) * nlen));
      }
      const V3 n2 = inside ? scale(nrm, -1.0) : nrm;
      const double r1 = inside ? 1.45 : 1.0, r2 = inside ? 1.0 : 1.45;
      bool tir = false;
      V3 tdir = {0.0, 0.0, 0.0};
      const bool do_refr = REFR && depth < max_depth && transp != 0.0;   // :242
      if (do_refr) tdir = refract_dir(rd, n2, r1 / r2, &tir);
      const double rp = tir ? refl + (1.0 - refl) * transp : refl;       // :261-265
      const bool do_refl = depth < max_depth && rp != 0.0 && (!inside || tir);   // :267
      if constexpr (POOL) {             // one push point for both kinds of child (see pool_push)
        const bool rfr = do_refr && !tir;
        if (rfr || do_refl) {
          const double w = rfr ? transp : rp;
          push_A = intensify<FC>(L, 1.0 - w);
          push_w = w;
          pushing = true;
        }
      }
      if (do_refr && !tir) {
        if constexpr (!POOL) put_frame(sp, intensify<FC>(L, 1.0 - transp), transp);
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
        if constexpr (!POOL) put_frame(sp, intensify<FC>(L, 1.0 - rp), rp);
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
    if constexpr (POOL) {                                                // frame `iter` (= sp before the push)
      if (iter < KL) {
        if (pushing) put_frame(iter, push_A, push_w);                     // the lane's own LDS slot
      } else {
        pool_push(pushing, iter, push_A, push_w, oi);
      }
    }
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

// REFR (scenes with RtDevScene::ray_chains and a transparent object): a hit spawns a refraction
// ray (weight transparency) or, on TIR or for a reflective object, a reflection ray (weight rp,
// raytracer.rs:261-265), never both, so the rays still form a chain and the same three phases
// apply; the decisions, directions and weights are trace<true, ..., CHAIN>'s, the traversals take
// the refraction kernels' template arguments (shared sphere terms, draw-order shadow walk: the
// transparency product's order is the reference's).
template <int HC, bool FC = false, bool REFR = false>
RT_FN Col trace_deferred(const DS& S, V3 ro, V3 rd, int max_depth, bool valid, ShadowWin* win) {
  constexpr bool SHARE = REFR && RT_SPHERE_SHARE, OBB = !REFR;
  double hP[HC][3], hN[HC][3], hC[HC][3], hW[HC];
  int nh = 0;
  bool last_spawned = false;          // the last hit spawned a reflection ray (that missed)
  // ---- phase 1: the nearest-hit chain
  if (valid) {
    for (int depth = 0;; ++depth) {
      double t_hit;
      const int oi = nearest_hit<SHARE, OBB>(S, ro, rd, &t_hit);
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
        RT_REC(lt, S, lights, LIGHTS, k);
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
  Col C = {0.0, 0.0, 0.0};
  for (int h = nh - 1; h >= 0; --h) {
    const Col L = {hC[h][0], hC[h][1], hC[h][2]};
    const double w = hW[h];
    C = (h == nh - 1 && !last_spawned) ? L : cadd<FC>(intensify<FC>(L, 1.0 - w), intensify<FC>(C, w));   // :278-279
  }
  return C;
}

// RT_SPEC: every table is the scene's constexpr copy (spec.hip), only the texels stay in HBM;
// RT_SPEC_FAMILY: the family's constexpr tables plus this scene's own (RT_REC).
__device__ __forceinline__ DS make_ds(const RtDevScene& s) {
  DS d;
#ifdef RT_SPEC
#ifdef RT_SPEC_FAMILY
  // the merged tables (RT_REC) read this scene's own; nodes, programs and textures are the family's
  d.objects = as_const(s.objects);
  d.trav = as_const(s.trav);
  d.strav = as_const(s.strav);
  d.leaves = as_const(s.leaves);
  d.lights = as_const(s.lights);
#else
  d.objects = as_const(rt_spec::OBJECTS);
  d.trav = as_const(rt_spec::TRAV);
  d.strav = as_const(rt_spec::STRAV);
  d.leaves = as_const(rt_spec::LEAVES);
  d.lights = as_const(rt_spec::LIGHTS);
#endif
  d.n_trav = rt_spec::N_TRAV;
  d.n_strav = rt_spec::N_STRAV;
  d.nodes = as_const(rt_spec::NODES);
  d.prog = as_const(rt_spec::PROG);
  d.textures = as_const(rt_spec::TEXTURES);
  d.n_objects = rt_spec::N_OBJECTS;
  d.n_lights = rt_spec::N_LIGHTS;
  d.shadow_early_out = rt_spec::SHADOW_EARLY_OUT;
#else
  d.objects = as_const(s.objects);
  d.trav = as_const(s.trav);
  d.n_trav = s.n_trav;
  d.strav = as_const(s.strav);
  d.n_strav = s.n_strav;
  d.trav_c = as_const(s.trav_c);
  d.strav_c = as_const(s.strav_c);
  d.nodes = as_const(s.nodes);
  d.leaves = as_const(s.leaves);
  d.prog = as_const(s.prog);
  d.lights = as_const(s.lights);
  d.textures = as_const(s.textures);
  d.n_objects = s.n_objects;
  d.n_lights = s.n_lights;
  d.shadow_early_out = s.shadow_early_out;
#endif
  d.texels = s.texels;
  return d;
}

// PerspectiveCamera::create_ray (camera.rs:65-74)
__device__ __forceinline__ void camera_ray(const RtCamera& cam, double x, double y, V3* ro, V3* rd) {
  double sx = ((x / cam.width) - 0.5) * cam.aspect;
  double sy = (cam.height - 1.0 - y) / cam.height - 0.5;
  *rd = add(add(ld3(cam.direction), scale(ld3(cam.right), sx)), scale(ld3(cam.up), sy));
  *ro = ld3(cam.center);
}

// The same ray for an integer pixel (x, y) in the frame: the two divisions and their terms read from
// the upload's per-column / per-row tables (RtDevScene::cam_sx / cam_sy, computed by the host with
// camera_ray's expressions), the rest as camera_ray.
__device__ __forceinline__ void camera_ray_px(const RtDevScene& S, int x, int y, V3* ro, V3* rd) {
  const double sx = S.cam_sx[x], sy = S.cam_sy[y];
  *rd = add(add(ld3(S.cam.direction), scale(ld3(S.cam.right), sx)), scale(ld3(S.cam.up), sy));
  *ro = ld3(S.cam.center);
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
// Tile = the 64 pixels of one wave, RT_TILE_W x RT_TILE_H (RT_TILE_W in rt_blob.h).  Pixel `pix` of tile `tile` -> (x, output row r).
constexpr int RT_TILE_H = 64 / RT_TILE_W;
static_assert(RT_TILE_W * RT_TILE_H == 64, "a tile is one wave's 64 pixels");
__device__ __forceinline__ void tile_pixel(unsigned tile, int pix, int width, int* x, int* r) {
  const unsigned tiles_x = (unsigned)(width + RT_TILE_W - 1) / RT_TILE_W;
  *x = (int)(tile % tiles_x) * RT_TILE_W + pix % RT_TILE_W;
  *r = (int)(tile / tiles_x) * RT_TILE_H + pix / RT_TILE_W;
}

// Output row r of a launch -> its frame row (see above); a launch of one band (every single-GPU frame)
// skips the per-lane integer division and remainder (a wave-uniform branch).
__device__ __forceinline__ int band_row(int r, int y_first, int band_rows, int band_pitch, int n_rows) {
  if (band_rows >= n_rows) return y_first + r;
  return y_first + (r / band_rows) * band_pitch + r % band_rows;
}

// One pixel's colour into an output row: f64 RGBA (alpha 1 after any colour op), packed RGB8 (band
// gathers) or RGBA8 with `(c * 255.0) as u8` per channel (easy_pixbuf.rs:46-53).
// The RGBA8 / RGB8 frame is written once and read by another kernel or the host: nontemporal
// (streaming) stores.  A wave's 8x8 tile covers a quarter of eight 128-byte lines and the tiles
// sharing a line run at different times on different XCDs, so through the L2s every row segment
// reached memory as its own partial-line write-back: WRITE_SIZE counted 118 MiB for a 31.6 MiB
// background-only 4K frame, 71 MiB with streaming stores, at equal kernel time
// (profiles/r06h_nt_stores.txt).  Diagnostic builds with RT_PLAIN_STORES keep plain stores.
// PLAIN: write-back stores (the primary-ray kernels, below).
template <bool PLAIN = false, class T>
__device__ __forceinline__ void frame_store(T v, T* p) {
#ifdef RT_PLAIN_STORES
  *p = v;
#else
  if constexpr (PLAIN) *p = v;
  else __builtin_nontemporal_store(v, p);
#endif
}
template <bool F64, bool PLAIN = false>
__device__ __forceinline__ void store_pixel(uint8_t* row, int x, Col c, int rgb) {
  if constexpr (F64) {
    double* o = (double*)row + (size_t)x * 4;
    o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = 1.0;
  } else if (rgb) {
    uint8_t* o = row + (size_t)x * 3;
    frame_store<PLAIN>((uint8_t)to_u8(c.r), o);
    frame_store<PLAIN>((uint8_t)to_u8(c.g), o + 1);
    frame_store<PLAIN>((uint8_t)to_u8(c.b), o + 2);
  } else {
    frame_store<PLAIN>(to_u8(c.r) | (to_u8(c.g) << 8) | (to_u8(c.b) << 16) | (255u << 24), (uint32_t*)row + x);
  }
}

// ---------------------------------------------------------------- kernel bodies
// The row kernels' bodies, shared by the generic kernels (k_rows.hip) and the scene-specialised ones
// (k_spec.hip).  Output rows r = 0 .. n_rows-1 of a band layout; wave = one 8x8 tile.
// Tile dispatch order (see launch_bands): `order` lists the tiles most expensive first, as measured
// on a calibration launch that stored each tile's wave time in `cost`.  CAL (the calibration
// instantiation) is the only one that carries the timing code.
// KL_ >= 0: that many stack frames in LDS (the specialised kernels at 4 waves/SIMD have room for more).
// rows_entry: entry `entry` of the launch (a tile index, or the order's entry-th tile); rows_body: the
// workgroup's own entry (blockIdx.x).  (A wave looping over several entries grid-stride was measured
// and lost: the loop's live state cost the megakernels 6 more spilled VGPRs, profiles/r07c_tiles_per_wave.txt.)
// The row kernels' frame storage per one-wave workgroup: the reflection-only and chain modes take a
// wave pool (trace(), KP slots) by default; KL_ >= 0 asks for KL_ frames per lane instead (the round-4
// layout, diagnostic A/B); KP_ >= 0 sets the pool's size.  The ray-tree mode keeps per-lane frames.
// Measured (profiles/r07g_pool_refl_ab.txt, r07h_hybrid_refl_ab.txt; anim120 bench lines r07e-r07h):
//   reflection-only, 4K globes: 2 per-lane frames 0.3215 ms, 114.7 MB of HBM per launch; a pool of 122
//     slots 0.3287 ms, 93.1 MB; 2 frames + a pool of 58: 0.3269 ms, 107.9 MB -- chains are short there,
//     and the pool's ballots and header reads cost more than the scratch they save: no pool;
//   chain, anim120 (Mrays/s, MB per 1080p frame): 5 per-lane frames (round 4, 10 KB: 4 waves/SIMD)
//     14 766 / 48.7; 1 per-lane frame 16 251-16 378 / 147.5; 2: 16 149 / 116.5; 1 frame + a pool of 122
//     (6 KB: 6 waves/SIMD with the family programs' 80 VGPRs) 16 061-16 095 / 93.4; pools of 186 / 250 /
//     314 slots 16 036 / 15 205 / 14 984 at 92.9 / 67.1 / 46.4 -- 1 frame + 122 is kept: the occupancy of
//     the fastest layout at 63 % of its traffic.
#ifndef RT_LDS_POOL_REFL
#define RT_LDS_POOL_REFL 0
#endif
//   round 6, pool slots of 25 B (RT_POOL_OBJ_INDEX), f32 culling (profiles/r09d_anim_pool_sweep.txt; anim120
//     Mrays/s, MB per 1080p frame): 1 per-lane frame + 122 slots 17 152 / 94.3; 1 + 183: 16 645 / 70.1;
//     1 + 238: 16 119 / 50.4; 0 + 265 (6.7 KB: 6 waves/SIMD) 16 660 / 61.2; 0 + 320 (8 KB: 5 waves/SIMD)
//     16 118 / 41.5 (FETCH 7.4 MiB) -- 0 + 320 is kept: the round-5 verdict's traffic bar (<= 48 MB per frame,
//     FETCH <= 8 MiB at >= 16 000 Mrays/s) at 6 % below the fastest layout.
#ifndef RT_LDS_POOL_CHAIN
#define RT_LDS_POOL_CHAIN 320       // no per-lane frame: 8 KB per one-wave workgroup, 20 per CU (5 waves/SIMD)
#endif
template <int MODE, int KL_ = -1, int KP_ = -1>
constexpr int rows_pool_slots() {
  return MODE == RT_MODE_TREE ? 0 : KP_ >= 0 ? KP_ : MODE == RT_MODE_CHAIN ? RT_LDS_POOL_CHAIN : RT_LDS_POOL_REFL;
}
template <int MODE, int KL_ = -1>
constexpr int rows_lane_frames() {
  return KL_ >= 0 ? KL_ : MODE == RT_MODE_CHAIN ? RT_LDS_FRAMES_CHAIN : RT_LDS_FRAMES;
}
// PRIM (the primary-ray kernels of the specialised programs, launches with max_depth 0): max_depth is the
// compile-time 0, so trace() never pushes a frame -- no frame stack, no LDS, no bounce loop -- and the
// frame takes write-back stores (such launches order their tiles by 128-byte line and XCD, k_rows.hip
// xcd_line_order, so a line's four tiles are written back to back through one L2).
template <int MODE, bool F64, bool CAL, bool FC, int KL_ = -1, int KP_ = -1, bool PRIM = false>
__device__ __forceinline__ void rows_entry(const RtDevScene& S, unsigned entry, int y_first, int band_rows, int band_pitch,
                                           int n_rows, int max_depth, uint8_t* __restrict__ out, size_t stride,
                                           const int32_t* __restrict__ order, uint32_t* __restrict__ cost, int rgb,
                                           lds_f64* frames) {
  constexpr bool REFR = MODE != RT_MODE_REFL, CHAIN = MODE == RT_MODE_CHAIN;
  constexpr int KLR = PRIM ? 0 : MODE == RT_MODE_TREE ? RT_LDS_RFRAMES : 0;
  constexpr int KP = PRIM ? 0 : rows_pool_slots<MODE, KL_, KP_>();
  constexpr int KL = PRIM ? 0 : rows_lane_frames<MODE, KL_>();
  if constexpr (PRIM) max_depth = 0;
  const int lane = threadIdx.x & 63;
  const unsigned tile = CAL || !order ? entry : (unsigned)order[entry];
  [[maybe_unused]] uint64_t t_start = 0;
  if constexpr (CAL) t_start = wall_clock64();
  int x, r;
  tile_pixel(tile, lane, S.width, &x, &r);
  if (x >= S.width || r >= n_rows) return;
  const int y = band_row(r, y_first, band_rows, band_pitch, n_rows);
  if (y >= S.height) return;
  V3 ro, rd;
  camera_ray_px(S, x, y, &ro, &rd);                                         // get_pixel(x as f64, y as f64)
  const Col c = trace<REFR, NoRec, KL, FC, KLR, CHAIN, KP>(make_ds(S), ro, rd, max_depth, nullptr, PRIM ? nullptr : frames + lane,
                                                         frames);
  store_pixel<F64, PRIM>(out + (size_t)r * stride, x, c, rgb);
  if constexpr (CAL)
    if (threadIdx.x == 0) cost[tile] = (uint32_t)(wall_clock64() - t_start);   // vector store
}
template <int MODE, bool F64, bool CAL, bool FC, int KL_ = -1, int KP_ = -1, bool PRIM = false>
__device__ __forceinline__ void rows_body(const RtDevScene& S, int y_first, int band_rows, int band_pitch, int n_rows,
                                          int max_depth, uint8_t* __restrict__ out, size_t stride,
                                          const int32_t* __restrict__ order, uint32_t* __restrict__ cost, int rgb,
                                          lds_f64* frames) {
  rows_entry<MODE, F64, CAL, FC, KL_, KP_, PRIM>(S, blockIdx.x, y_first, band_rows, band_pitch, n_rows, max_depth, out,
                                                 stride, order, cost, rgb, frames);
}
template <int MODE, int KL_ = -1, int KP_ = -1>
constexpr int rows_lds_doubles() {
  return (rows_lane_frames<MODE, KL_>() * 4 + (MODE == RT_MODE_TREE ? RT_LDS_RFRAMES : 0) * 7) * 64 +
         (rows_pool_slots<MODE, KL_, KP_>() > 0
              ? RT_POOL_HDR + pool_doubles<rows_pool_slots<MODE, KL_, KP_>(), RT_POOL_OBJ_INDEX != 0>()
              : 0);
}

// The deferred-shadow kernel's body (reflection-only scenes, or refraction chains on request): one
// wave per 8x8 tile, every tile on the deferred path (trace_deferred), and the costliest tiles split
// over P = 2, 4 or 8 waves: wave `part` renders pixels [part * 64/P, (part + 1) * 64/P) of the tile
// on its first 64/P lanes and its other lanes only trace shadow rays (phase 2).  Order entry:
// tile | part << 20 | log2(P) << 24 (built by launch_bands after the calibration launch).
template <bool F64, bool CAL, bool FC, bool REFR>
__device__ __forceinline__ void deferred_body(const RtDevScene& S, int y_first, int band_rows, int band_pitch,
                                              int n_rows, int max_depth, uint8_t* __restrict__ out, size_t stride,
                                              const int32_t* __restrict__ order, uint32_t* __restrict__ cost, int rgb,
                                              ShadowWin* win) {
  const int lane = threadIdx.x & 63;
  const uint32_t e = CAL || !order ? blockIdx.x : (uint32_t)order[blockIdx.x];
  const unsigned tile = e & RT_SPLIT_TILE_MASK;
  const int lp = (int)((e >> 24) & 7u), per = 64 >> lp;
  const int pix = (int)((e >> 20) & 15u) * per + lane;
  [[maybe_unused]] uint64_t t_start = 0;
  if constexpr (CAL) t_start = wall_clock64();
  int x, r;
  tile_pixel(tile, pix, S.width, &x, &r);
  int y = 0;
  bool valid = lane < per && x < S.width && r < n_rows;
  if (valid) {
    y = band_row(r, y_first, band_rows, band_pitch, n_rows);
    valid = y < S.height;
  }
  V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
  if (valid) camera_ray_px(S, x, y, &ro, &rd);                              // get_pixel(x as f64, y as f64)
  const Col c = trace_deferred<RT_MAX_DEPTH_CAP + 1, FC, REFR>(make_ds(S), ro, rd, max_depth, valid, win);
  if (valid) store_pixel<F64>(out + (size_t)r * stride, x, c, rgb);
  if constexpr (CAL)
    if (lane == 0) cost[tile] = (uint32_t)(wall_clock64() - t_start);
}
#ifndef RT_WAVES_PER_EU_DEFERRED
#define RT_WAVES_PER_EU_DEFERRED 7
#endif

}  // namespace
