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
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#define RT_HD __device__
#include "rt_blob.h"
#include "rt_math.h"
#include "scene.h"

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

namespace {

// Scene tables are read-only for the whole launch: view them through the CONSTANT address space
// (4) so uniform-index reads compile to scalar (SMEM) loads instead of per-lane VMEM loads.
#define CAS __attribute__((address_space(4)))
template <class T> using cptr = const CAS T*;
template <class T> __device__ __forceinline__ cptr<T> as_const(const T* p) { return (cptr<T>)p; }

struct DS {                         // device view of RtDevScene
  cptr<RtObject> objects;
  cptr<RtNode> nodes;
  cptr<RtLeaf> leaves;
  cptr<RtProg> prog;
  cptr<RtLight> lights;
  cptr<RtTexture> textures;
  const uint8_t* texels;            // per-lane texel gathers stay global (vector) loads
  int n_objects, n_lights;
  int shadow_early_out;
};

constexpr double EPS = RT_EPSILON;
#define RT_LIGHT_GROUP 4            // shadow transparencies held in registers per light group
constexpr double PI_D = 3.14159265358979323846;   // std::f64::consts::PI

struct V3 { double x, y, z; };
struct Col { double r, g, b; };

__device__ __forceinline__ V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 scale(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double len(V3 a) { return sqrt(dot(a, a)); }
__device__ __forceinline__ V3 normalized(V3 a) { return scale(a, 1.0 / len(a)); }
template <class P> __device__ __forceinline__ V3 ld3(P p) { return {p[0], p[1], p[2]}; }
// transform_vector (transformation.rs:53-59) with rows m[0..3], m[4..7], m[8..11]
template <class P> __device__ __forceinline__ V3 xf(P m, V3 v) {
  return {m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3],
          m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7],
          m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11]};
}
// color.rs:36-53: clamp each channel (NaN passes through)
__device__ __forceinline__ double in_limit(double x) { return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x); }
__device__ __forceinline__ Col in_range(double r, double g, double b) { return {in_limit(r), in_limit(g), in_limit(b)}; }
__device__ __forceinline__ Col intensify(Col c, double k) { return in_range(c.r * k, c.g * k, c.b * k); }
__device__ __forceinline__ Col cmul(Col a, Col b) { return in_range(a.r * b.r, a.g * b.g, a.b * b.b); }
__device__ __forceinline__ Col cadd(Col a, Col b) { return in_range(a.r + b.r, a.g + b.g, a.b + b.b); }
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

__device__ bool leaf_inside(cptr<RtLeaf> L, V3 p) {
  int k = L->kind;
  if (k == RT_N_PLANE) return false;                                        // :186-188
  V3 q = xf(L->inv, p);
  if (k == RT_N_SPHERE) return len(sub(q, ld3(L->c))) <= L->r_eps;         // :70-74
  return q.x <= L->hi[0] && q.x >= L->lo[0] && q.y <= L->hi[1] &&          // :319-328
         q.y >= L->lo[1] && q.z <= L->hi[2] && q.z >= L->lo[2];
}

__device__ bool leaf_on_surface(cptr<RtLeaf> L, V3 p) {
  V3 q = xf(L->inv, p);
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

__device__ V3 leaf_normal(cptr<RtLeaf> L, V3 p) {
  int k = L->kind;
  if (k == RT_N_PLANE) return ld3(L->pn[0]);                               // :182-184
  V3 q = xf(L->inv, p);
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
  V3 q = xf(L->inv, sub(p, ld3(L->c)));
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
__device__ __forceinline__ int leaf_candidates(cptr<RtLeaf> L, V3 ro, V3 rd, double* t0, double* t1) {
  V3 o = xf(L->inv, ro);                                                   // transformation.rs:88-93
  V3 d = sub(xf(L->inv, rd), ld3(L->inv_o));
  int k = L->kind;
  if (k == RT_N_SPHERE) {                                                  // math_shapes.rs:42-62
    V3 v = sub(o, ld3(L->c));
    double il = 1.0 / len(d);
    V3 dn = scale(d, il);
    double vd = dot(v, dn);
    double sum = vd * vd - (dot(v, v) - L->r2);
    if (sum < 0.0) return 0;
    double sq = sqrt(sum);
    *t0 = (-vd + sq) * il;
    *t1 = (-vd - sq) * il;
    return 2;
  }
  if (k == RT_N_PLANE) {                                                   // :168-180
    V3 pn = ld3(L->pnorm);
    double v_d = dot(pn, d);
    if (v_d != 0.0) {
      double t = -(dot(pn, o) + L->pl[0][3]) * (1.0 / v_d);
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
  uint32_t st = 0;
  const int e = L->prog_end;
  for (int k = L->prog_begin; k < e; ++k) {
    const int op = S.prog[k].op, arg = S.prog[k].arg;
    if (op == RT_OP_INSIDE) {
      st = (st << 1) | (leaf_inside(&S.leaves[arg], p) ? 1u : 0u);
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
// Does the ray segment t in [0, tmax] come near the box?  Only ever answers "no" when no point of
// the segment is inside [lo, hi]; boxes are inflated on the host (scene.cpp leaf_box) and tmax
// carries a relative margin, so f64 rounding here cannot cull a hit the exact code would accept.
// NaN anywhere makes the comparisons false and the answer "yes" (evaluate exactly).
template <class P> __device__ __forceinline__ bool box_may_hit(P lo, P hi, V3 o, V3 d, V3 inv, double tmax) {
#ifndef RT_BRANCHY_BOX
  // Select form (no exec-mask branches).  An axis with d == 0 only asks whether the origin lies
  // in the slab; otherwise the usual interval narrowing, where a NaN bound narrows nothing.
  double tn = 0.0, tf = tmax;
  bool out = false;
#define RT_BOXAX(P, D, I, IV)                                                   \
  {                                                                             \
    const double a = (lo[I] - P) * IV, b = (hi[I] - P) * IV;                    \
    const bool z = D == 0.0;                                                    \
    out = out || (z && (P < lo[I] || P > hi[I]));                               \
    const bool sw = a > b;                                                      \
    const double mn = sw ? b : a, mx = sw ? a : b;                              \
    tn = (!z && mn > tn) ? mn : tn;                                             \
    tf = (!z && mx < tf) ? mx : tf;                                             \
  }
  RT_BOXAX(o.x, d.x, 0, inv.x)
  RT_BOXAX(o.y, d.y, 1, inv.y)
  RT_BOXAX(o.z, d.z, 2, inv.z)
#undef RT_BOXAX
  return !out && !(tn > tf);
#else
  double tn = 0.0, tf = tmax;
#define RT_BOXAX(P, D, I, IV)                                                   \
  if (D == 0.0) {                                                               \
    if (P < lo[I] || P > hi[I]) return false;                                   \
  } else {                                                                      \
    double a = (lo[I] - P) * IV, b = (hi[I] - P) * IV;                          \
    if (a > b) { double tmp = a; a = b; b = tmp; }                              \
    if (a > tn) tn = a;                                                         \
    if (b < tf) tf = b;                                                         \
  }
  RT_BOXAX(o.x, d.x, 0, inv.x)
  RT_BOXAX(o.y, d.y, 1, inv.y)
  RT_BOXAX(o.z, d.z, 2, inv.z)
#undef RT_BOXAX
  return !(tn > tf);
#endif
}
// Reciprocal for the culling slabs only (never for a value the reference computes): hardware
// rcp + one Newton step, ~1e-15 relative -- far inside the culling margins.  d == 0 -> NaN or
// inf, which box_may_hit never reads (that axis takes the d == 0 branch).
__device__ __forceinline__ double cull_rcp(double x) {
#ifdef RT_EXACT_CULL_RCP
  return 1.0 / x;
#else
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
#endif
}
__device__ __forceinline__ V3 cull_inv(V3 d) { return {cull_rcp(d.x), cull_rcp(d.y), cull_rcp(d.z)}; }
__device__ __forceinline__ double cull_tmax(double t) { return t * (1.0 + 1e-7) + 1e-7; }

// ------------------------------------------------------------------ traversal (raytracer.rs)
// Nearest hit over all objects in draw order: accept d if d > EPS && d < nearest
// (raytracer.rs:141-150).  The acceptance test is pure, so it runs BEFORE the (pure) CSG
// filter: candidates that cannot win never pay for the sibling is_inside tests.
__device__ int nearest_hit(const DS& S, V3 ro, V3 rd, double* dist) {
  double best = INFINITY;
  int bobj = -1;
  const V3 inv = cull_inv(rd);
  for (int o = 0; o < S.n_objects; ++o) {
    cptr<RtObject> O = &S.objects[o];
    if (O->cull == RT_CULL_ALWAYS) continue;
    if (O->cull == RT_CULL_BOX && !box_may_hit(O->blo, O->bhi, ro, rd, inv, cull_tmax(best))) continue;
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    for (int l = lb; l < le; ++l) {
      cptr<RtLeaf> L = &S.leaves[l];
      if (O->leaf_cull) {
        if (L->cull == RT_CULL_ALWAYS) continue;
        if (L->cull == RT_CULL_BOX && !box_may_hit(L->blo, L->bhi, ro, rd, inv, cull_tmax(best))) continue;
      }
      double t0 = 0.0, t1 = 0.0;
      int n = leaf_candidates(L, ro, rd, &t0, &t1);
      const bool filtered = L->prog_end != L->prog_begin;
      if (n >= 1 && t0 > EPS && t0 < best && (!filtered || leaf_filter(S, L, add(ro, scale(rd, t0))))) {
        best = t0; bobj = o;
      }
      if (n >= 2 && t1 > EPS && t1 < best && (!filtered || leaf_filter(S, L, add(ro, scale(rd, t1))))) {
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
__device__ double shadow_transparency(const DS& S, V3 p, V3 dir, double dist) {
  double tr = 1.0;
  const V3 inv = cull_inv(dir);
  const double tmax = cull_tmax(dist);
  for (int o = 0; o < S.n_objects; ++o) {
    cptr<RtObject> O = &S.objects[o];
    if (O->shadow_skip || O->cull == RT_CULL_ALWAYS) continue;
    if (O->cull == RT_CULL_BOX && !box_may_hit(O->blo, O->bhi, p, dir, inv, tmax)) continue;
    const double tobj = O->transparency;
    const int lb = O->leaf_begin, le = lb + O->leaf_count;
    for (int l = lb; l < le; ++l) {
      cptr<RtLeaf> L = &S.leaves[l];
      if (O->leaf_cull) {
        if (L->cull == RT_CULL_ALWAYS) continue;
        if (L->cull == RT_CULL_BOX && !box_may_hit(L->blo, L->bhi, p, dir, inv, tmax)) continue;
      }
      double t0 = 0.0, t1 = 0.0;
      int n = leaf_candidates(L, p, dir, &t0, &t1);
      const bool filtered = L->prog_end != L->prog_begin;
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
  *u = 0.0;
  *v = 0.0;
  if (cnt == 1) {
    cptr<RtLeaf> L = &S.leaves[N[0].leaf];
    *n = leaf_normal(L, p);
    if (want_uv && L->kind == RT_N_SPHERE) sphere_uv(L, p, u, v);
    return;
  }
  uint32_t in = 0, on = 0;
  for (int i = 0; i < cnt; ++i) {
    const int nk = N[i].kind, na = N[i].a, nb = N[i].b, nl = N[i].leaf;
    bool bi, bo;
    if (nk < RT_N_UNION) {
      cptr<RtLeaf> L = &S.leaves[nl];
      bi = leaf_inside(L, p);
      bo = leaf_on_surface(L, p);
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
    *n = leaf_normal(L, p);
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

__device__ __forceinline__ V3 reflect_dir(V3 i, V3 n) {                    // raytracer.rs:332-334
  return sub(i, scale(scale(n, 2.0), dot(n, i)));
}
__device__ __forceinline__ V3 refract_dir(V3 i, V3 n, double r, bool* tir) {   // raytracer.rs:336-353
  double cos_1 = dot(scale(i, -1.0), n);
  double v = 1.0 - r * r * (1.0 - cos_1 * cos_1);
  *tir = v < 0.0;
  if (*tir) return {0.0, 0.0, 0.0};
  double cos_2 = sqrt(v);
  return normalized(add(scale(i, r), scale(n, r * cos_1 - cos_2)));
}

// Normal (normalised, :163), material colour at the UV (:165-170), transparency, reflectivity of
// each lane's hit object -- SCALARISED over the distinct objects hit in this wave (readlane of the
// first remaining lane), so every object / node / leaf read is wave-uniform (SMEM, no VGPRs).
__device__ __forceinline__ void shade_inputs(const DS& S, int oi, V3 p, V3* nrm, Col* c, double* transp,
                                             double* refl) {
  uint64_t todo = __ballot(oi >= 0);
  while (todo) {
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

// get_ray_color (raytracer.rs:132-287) for one primary ray, recursion unrolled onto a per-lane
// frame stack.  REFR = the scene has a transparent object (refraction frames need more state).
template <bool REFR>
__device__ Col trace(const DS& S, V3 ro, V3 rd, int max_depth) {
  double fA[RT_MAX_DEPTH_CAP][3];     // parent colour already intensified by (1 - w)
  double fW[RT_MAX_DEPTH_CAP];        // child weight w (transparency or reflectivity)
  double fP[REFR ? RT_MAX_DEPTH_CAP : 1][3], fD[REFR ? RT_MAX_DEPTH_CAP : 1][3];
  double fRP[REFR ? RT_MAX_DEPTH_CAP : 1];
  int fPend[REFR ? RT_MAX_DEPTH_CAP : 1];
  int sp = 0, depth = 0;
  Col C = {0.0, 0.0, 0.0};
  [[maybe_unused]] int trip = 0;
  for (;;) {
    bool descend = false;
    double t_hit;
    PROF_T0(p0);
    const int oi = nearest_hit(S, ro, rd, &t_hit);
    PROF_ADD(trip == 0 ? 0 : 1, p0);
    ++trip;
    PROF_T0(p1);
#ifdef RT_ABLATE_TRAVERSAL_ONLY          // diagnostic builds only (tools/ablation): cost split
    return Col{t_hit * 1e-3, (double)oi, 0.0};
#endif
    const V3 p = add(ro, scale(rd, t_hit));                               // :162
    V3 nrm = {0.0, 0.0, 0.0};
    Col c = {0.0, 0.0, 0.0}, L = {0.0, 0.0, 0.0};
    double transp = 0.0, refl = 0.0;
    if (oi >= 0) {
      // Evaluation order is free (every step is a pure function of the hit), so the shadow
      // rays of a group of lights are traced FIRST, while only the hit point is live, and the
      // normal / UV / material and the per-light Lambert terms are formed afterwards: far fewer
      // registers live across the traversals.  Light accumulation order is unchanged.
      bool have_shading = false;
      for (int base = 0; base < S.n_lights; base += RT_LIGHT_GROUP) {
        double tr[RT_LIGHT_GROUP];
#pragma unroll
        for (int k = 0; k < RT_LIGHT_GROUP; ++k) tr[k] = 0.0;
        const int nk = S.n_lights - base < RT_LIGHT_GROUP ? S.n_lights - base : RT_LIGHT_GROUP;
#pragma unroll 1
        for (int k = 0; k < nk; ++k) {                                   // ONE traversal body in the code
          const V3 lv = sub(ld3(S.lights[base + k].p), p);
#ifdef RT_ABLATE_NO_SHADOWS
          const double t = lv.x > 1e300 ? 0.5 : 1.0;
#else
          PROF_T0(p2);
          const double t = shadow_transparency(S, p, normalized(lv), len(lv));   // :176-197
          PROF_ADD(2, p2);
#endif
#pragma unroll
          for (int j = 0; j < RT_LIGHT_GROUP; ++j) tr[j] = j == k ? t : tr[j];   // registers, no scratch
        }
        if (!have_shading) {
          PROF_T0(p3);
          shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);
          PROF_ADD(3, p3);
          L = cmul(c, in_range(0.6, 0.6, 0.6));                           // ambient (:172)
          have_shading = true;
        }
#pragma unroll
        for (int k = 0; k < RT_LIGHT_GROUP; ++k) {                       // :199-227
          if (base + k >= S.n_lights || tr[k] == 0.0) continue;
          cptr<RtLight> lt = &S.lights[base + k];
          const V3 sdir = normalized(sub(ld3(lt->p), p));
          double ang = rt_acos(dot(sdir, nrm) / (len(sdir) * len(nrm)));
          if (ang >= PI_D / 2.0) ang = PI_D - ang;
          const double inten = (ang < (PI_D / 2.0) && ang >= 0.0) ? 1.0 - (ang / (PI_D / 2.0)) : 0.0;
          const Col lc = intensify(intensify(Col{lt->col[0], lt->col[1], lt->col[2]}, inten), tr[k]);
          L = cadd(L, cmul(c, lc));
        }
      }
      if (!have_shading) {
        shade_inputs(S, oi, p, &nrm, &c, &transp, &refl);
        L = cmul(c, in_range(0.6, 0.6, 0.6));
      }
    }
    if (oi < 0) {
      C = {0.0, 0.0, 0.0};                                               // Color::BLACK (:152-160)
    } else {
      const V3 nd = scale(rd, -1.0);                                      // :230-235
      // angle(-dir, n) >= PI/2 (:230-231).  acos is monotone and rt_acos is within 1 ulp, so for
      // |cos| > 1e-15 (>= 4 ulp of PI/2 away from the threshold) the sign of the cosine decides
      // exactly; only near-grazing hits (and NaN) evaluate the acos itself.
      const double cin = dot(nd, nrm) / (len(nd) * len(nrm));
      const bool inside = cin < -1e-15 ? true : (cin > 1e-15 ? false : rt_acos(cin) >= PI_D / 2.0);
      const V3 n2 = inside ? scale(nrm, -1.0) : nrm;
      const double r1 = inside ? 1.45 : 1.0, r2 = inside ? 1.0 : 1.45;
      bool tir = false;
      V3 tdir = {0.0, 0.0, 0.0};
      const bool do_refr = REFR && depth < max_depth && transp != 0.0;   // :242
      if (do_refr) tdir = refract_dir(rd, n2, r1 / r2, &tir);
      const double rp = tir ? refl + (1.0 - refl) * transp : refl;       // :261-265
      const bool do_refl = depth < max_depth && rp != 0.0 && (!inside || tir);   // :267
      if (do_refr && !tir) {
        Col A = intensify(L, 1.0 - transp);
        fA[sp][0] = A.r; fA[sp][1] = A.g; fA[sp][2] = A.b;
        fW[sp] = transp;
        if constexpr (REFR) {
          fPend[sp] = do_refl ? 1 : 0;
          if (do_refl) {
            V3 rdir = reflect_dir(rd, n2);
            fP[sp][0] = p.x; fP[sp][1] = p.y; fP[sp][2] = p.z;
            fD[sp][0] = rdir.x; fD[sp][1] = rdir.y; fD[sp][2] = rdir.z;
            fRP[sp] = rp;
          }
        }
        ++sp;
        ro = p;
        rd = tdir;
        depth = sp;
        descend = true;
      } else if (do_refl) {
        Col A = intensify(L, 1.0 - rp);
        fA[sp][0] = A.r; fA[sp][1] = A.g; fA[sp][2] = A.b;
        fW[sp] = rp;
        if constexpr (REFR) fPend[sp] = 0;
        ++sp;
        rd = reflect_dir(rd, n2);
        ro = p;
        depth = sp;
        descend = true;
      } else {
        C = L;
      }
    }
    PROF_ADD(4, p1);
    if (descend) continue;
    while (sp > 0) {                                                      // post-order combine
      const int f = sp - 1;
      const Col comb = cadd(Col{fA[f][0], fA[f][1], fA[f][2]}, intensify(C, fW[f]));
      if constexpr (REFR) {
        if (fPend[f]) {                                                   // refraction done -> reflection
          fPend[f] = 0;
          Col A = intensify(comb, 1.0 - fRP[f]);
          fA[f][0] = A.r; fA[f][1] = A.g; fA[f][2] = A.b;
          fW[f] = fRP[f];
          ro = {fP[f][0], fP[f][1], fP[f][2]};
          rd = {fD[f][0], fD[f][1], fD[f][2]};
          depth = sp;
          descend = true;
          break;
        }
      }
      C = comb;
      --sp;
    }
    if (!descend) return C;
  }
}

__device__ __forceinline__ DS make_ds(const RtDevScene& s) {
  DS d;
  d.objects = as_const(s.objects);
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
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 4   // 128 VGPRs: measured best (profiles/r01_occupancy_sweep.txt)
#endif
template <bool REFR, bool F64>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU))) void render_rows_kernel(RtDevScene S, int y_first, int band_rows, int band_pitch,
                                                          int n_rows, int max_depth, uint8_t* __restrict__ out,
                                                          size_t stride) {
#ifdef RT_DIAG_LDS                       // diagnostic builds only: cap occupancy with an LDS pad
  __shared__ volatile char rt_pad[RT_DIAG_LDS];
  if (threadIdx.x == 0) rt_pad[0] = 0;
#endif
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_x = (S.width + 15) >> 4;
  const int bx = blockIdx.x % tiles_x, by = blockIdx.x / tiles_x;
  const int x = (bx << 4) + ((wave & 1) << 3) + (lane & 7);
  const int r = (by << 4) + ((wave >> 1) << 3) + (lane >> 3);
  if (x >= S.width || r >= n_rows) return;
  const int y = y_first + (r / band_rows) * band_pitch + r % band_rows;
  if (y >= S.height) return;
  V3 ro, rd;
  PROF_T0(p5);
  camera_ray(S.cam, (double)x, (double)y, &ro, &rd);                       // get_pixel(x as f64, y as f64)
  const Col c = trace<REFR>(make_ds(S), ro, rd, max_depth);
  PROF_ADD(5, p5);
  uint8_t* row = out + (size_t)r * stride;
  if constexpr (F64) {
    double* o = (double*)row + (size_t)x * 4;
    o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = 1.0;                        // alpha is 1 after any colour op
  } else {
    ((uint32_t*)row)[x] = to_u8(c.r) | (to_u8(c.g) << 8) | (to_u8(c.b) << 16) | (255u << 24);
  }
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

}  // namespace

// ====================================================================== device context
struct rt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;       // last stream launched on (NULL = the default stream)
  void* d_blob = nullptr;
  size_t blob_bytes = 0;
  RtDevScene dev;
  int32_t max_depth = 10;
  bool uploaded = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
};

using rt::fail;

#define RT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

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
  rt_ctx* c = new rt_ctx();
  c->device = device;
  memset(&c->dev, 0, sizeof c->dev);
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
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
  size_t o_obj = put(blob, f.objects), o_nodes = put(blob, f.nodes), o_leaves = put(blob, f.leaves);
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
  d.cam = f.cam;
  c->max_depth = f.max_depth;
  c->uploaded = true;
  return RT_OK;
}

static int launch_bands(rt_ctx* c, uint32_t y_first, uint32_t band_rows, uint32_t band_pitch, uint32_t n_bands,
                        int32_t max_depth, void* out, size_t stride, void* stream, bool f64) {
  if (!c || !out) return fail(RT_ERR_INVALID, "null argument");
  if (!c->uploaded) return fail(RT_ERR_INVALID, "no scene uploaded to this context");
  if (band_rows == 0 || n_bands == 0) return RT_OK;
  if (band_pitch < band_rows && n_bands > 1) return fail(RT_ERR_INVALID, "band pitch %u < band rows %u", band_pitch, band_rows);
  if (y_first >= (uint32_t)c->dev.height) return fail(RT_ERR_INVALID, "first row %u >= height %d", y_first, c->dev.height);
  const uint64_t n_rows64 = (uint64_t)band_rows * n_bands;
  if (n_rows64 > (1u << 24)) return fail(RT_ERR_INVALID, "too many rows");
  const uint32_t n_rows = (uint32_t)n_rows64;
  size_t row_bytes = (size_t)c->dev.width * (f64 ? 32 : 4);
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
  const int tiles_x = (c->dev.width + 15) / 16, tiles_y = (int)((n_rows + 15) / 16);
  dim3 grid((unsigned)(tiles_x * tiles_y)), block(256);
  const int a0 = (int)y_first, a1 = (int)band_rows, a2 = (int)band_pitch, a3 = (int)n_rows;
  RT_HIP(hipEventRecord(c->ev0, st));
  const bool refr = c->dev.any_transparent != 0;
  if (refr && f64) hipLaunchKernelGGL((render_rows_kernel<true, true>), grid, block, 0, st, c->dev, a0, a1, a2, a3, max_depth, target, tstride);
  else if (refr) hipLaunchKernelGGL((render_rows_kernel<true, false>), grid, block, 0, st, c->dev, a0, a1, a2, a3, max_depth, target, tstride);
  else if (f64) hipLaunchKernelGGL((render_rows_kernel<false, true>), grid, block, 0, st, c->dev, a0, a1, a2, a3, max_depth, target, tstride);
  else hipLaunchKernelGGL((render_rows_kernel<false, false>), grid, block, 0, st, c->dev, a0, a1, a2, a3, max_depth, target, tstride);
  RT_HIP(hipGetLastError());
  RT_HIP(hipEventRecord(c->ev1, st));
  c->timed = true;
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

int rt_render_rows(rt_ctx* c, uint32_t y0, uint32_t y1, int32_t max_depth, uint8_t* rgba8,
                   size_t row_stride_bytes, void* stream) {
  return launch_rows(c, y0, y1, max_depth, rgba8, row_stride_bytes, stream, false);
}

int rt_render_rows_f64(rt_ctx* c, uint32_t y0, uint32_t y1, int32_t max_depth, double* rgba,
                       size_t row_stride_bytes, void* stream) {
  return launch_rows(c, y0, y1, max_depth, rgba, row_stride_bytes, stream, true);
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
  RT_HIP(hipEventRecord(c->ev0, st));
  if (c->dev.any_transparent) hipLaunchKernelGGL((render_points_kernel<true>), grid, block, 0, st, c->dev, in, n, max_depth, target);
  else hipLaunchKernelGGL((render_points_kernel<false>), grid, block, 0, st, c->dev, in, n, max_depth, target);
  RT_HIP(hipGetLastError());
  RT_HIP(hipEventRecord(c->ev1, st));
  c->timed = true;
  if (!dev_out) {
    RT_HIP(hipMemcpyAsync(out, target, n * 4 * sizeof(double), hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
  }
  return RT_OK;
}

int rt_ctx_last_kernel_ms(rt_ctx* c, float* ms) {
  if (!c || !ms) return fail(RT_ERR_INVALID, "null argument");
  if (!c->timed) return fail(RT_ERR_INVALID, "no launch recorded");
  RT_HIP(hipEventSynchronize(c->ev1));
  RT_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
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
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  delete c;
}

}  // extern "C"
