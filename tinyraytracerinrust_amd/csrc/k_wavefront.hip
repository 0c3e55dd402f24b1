// k_wavefront.hip -- the wavefront path (one recursion depth per pass over a dense level of rays)
// and its pair path ((ray, object) work items sorted by object), launch-wide secondary-ray
// compaction for ray-tree scenes (DESIGN.md §2 "Wavefront path").  get_ray_color's operations per
// ray are rt_device.h's; this file reorganises WHEN they run, never what they compute.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "rt_device.h"
#include "rt_ctx.h"

namespace {

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
//   wf_fold_kernel   after every level is traced, from the deepest level up (RT_WF_FOLD_SPAN levels
//                    per launch): a ray's colour from its hit record and its children's colours:
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
  tile_pixel(slot >> 6, (int)(slot & 63), S.width, x, r);
  if (*x >= S.width || *r >= n_rows) return false;
  *y = band_row(*r, y_first, band_rows, band_pitch, n_rows);
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
      [&](double* t) { return *hit_obj = nearest_hit<SHARE, OBB>(S, ro, rd, t); },
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

#ifndef RT_WF_FOLD_SPAN
#define RT_WF_FOLD_SPAN 3                // levels folded per launch (1..3)
#endif
static_assert(RT_WF_FOLD_SPAN >= 1 && RT_WF_FOLD_SPAN <= 3, "fold span");
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
    if (live) camera_ray_px(S, x, y, &ro, &rd);                          // get_pixel(x as f64, y as f64)
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

// The folded colour of ray i of level d: its hit record and its children's colours -- computed here
// for the SPAN - 1 levels below d (a child has one parent: nothing is computed twice), read as stored
// (already folded) at level d + SPAN.  The same operations in the same order as one fold per level.
template <int SPAN, bool FC>
__device__ __forceinline__ Col wf_fold_node(const WfArena& A, int d, uint32_t i) {
  const WfLevel lv = wf_level(A, d);
  const Col L = {lv.Lr[i], lv.Lg[i], lv.Lb[i]};
  const int32_t ct = lv.ct[i], cr = lv.cr[i];
  auto child = [&](int32_t c) -> Col {
    if constexpr (SPAN > 1) {
      return wf_fold_node<SPAN - 1, FC>(A, d + 1, (uint32_t)c);
    } else {
      const WfLevel ch = wf_level(A, d + 1);
      return Col{ch.Lr[c], ch.Lg[c], ch.Lb[c]};
    }
  };
  Col C = L;
  if (ct >= 0) {                                             // refraction, then a pending reflection
    const double t = lv.wt[i];
    C = cadd<FC>(intensify<FC>(L, 1.0 - t), intensify<FC>(child(ct), t));
  }
  if (cr >= 0) {
    const double w = lv.wr[i];
    C = cadd<FC>(intensify<FC>(C, 1.0 - w), intensify<FC>(child(cr), w));
  }
  return C;
}

// Folds SPAN levels per launch (d .. d + SPAN - 1; level d's colours stored, or level 0's written as
// pixels): one launch boundary per SPAN levels (a boundary costs ~5 us on the pair path's small levels).
template <int SPAN, bool F64, bool FC>
__global__ __launch_bounds__(256) void wf_fold_kernel(RtDevScene S, WfArena A, int d, uint32_t n, const uint32_t* n_dev,
                                                      int y_first, int band_rows, int band_pitch, int n_rows,
                                                      uint8_t* __restrict__ out, size_t stride, int rgb) {
  if (n_dev) n = min(*n_dev, A.cap);                         // a device-driven level's count
  const WfLevel lv = wf_level(A, d);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int x = 0, r = 0, y = 0;
    if (d == 0 && (!wf_pixel(S, i, y_first, band_rows, band_pitch, n_rows, &x, &r, &y) || A.ovf[i])) continue;
    const Col C = wf_fold_node<SPAN, FC>(A, d, i);
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
    camera_ray_px(S, x, y, &ro, &rd);
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
                                //   grows the arena and runs the level again); [2]: a count passed 2^31
  uint32_t* bins;               // bucket-sort scratch: RT_WFP_BIN_WORDS words per sort
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
constexpr uint32_t RT_WFP_BIN_WORDS = 4096;   // one bucket sort's scratch (wf_sort.hip: counts + run cursors)
static_assert(RT_MAX_DEPTH_CAP + 3 <= RT_WFP_COUNT, "wavefront counter block");
static_assert(RT_WFP_COUNT + 5 <= 64, "wavefront counter block: 256 bytes");

// The object's nearest accepted distance for one ray: nearest_hit's body for one object, its best
// starting at +inf (the leaf boxes' tmax only shrinks, as share_prev requires).
__device__ __forceinline__ double wfp_object_nearest(const DS& S, int o, V3 ro, V3 rd, const CullR& cr) {
  const bool cf_ok = RT_CONST_FILTER && const_filter_range(ro, rd);
  cptr<RtObject> O = &S.objects[o];
  const bool fin = wave_finite(ro, rd);
  double best = INFINITY;
  SphereShare shr = {0.0, 0.0, 0.0};
  const int lb = O->leaf_begin, le = lb + O->leaf_count;
  for (int l = lb; l < le; ++l) {
    cptr<RtLeaf> L = &S.leaves[l];
    if (O->leaf_cull) {
      if (L->cull == RT_CULL_ALWAYS) continue;
      if (L->cull == RT_CULL_BOX && !RT_BOX_MAY_HIT(L, blo, bhi, cr, RT_CULL_TMAX(best))) continue;
    }
    double t0 = 0.0, t1 = 0.0;
    const int n = leaf_candidates<true>(L, ro, rd, fin, &t0, &t1, RT_SPHERE_SHARE ? &shr : nullptr);
    const bool filtered = L->prog_end != L->prog_begin && !(cf_ok && L->filter_const);
    if (n >= 1 && t0 > EPS && t0 < best && (!filtered || leaf_filter(S, L, add(ro, scale(rd, t0))))) best = t0;
    if (n >= 2 && t1 > EPS && t1 < best && (!filtered || leaf_filter(S, L, add(ro, scale(rd, t1))))) best = t1;
  }
  return best;
}

// Filtered hits of the object with EPS < t < dist on one shadow ray (shadow_transparency's body for
// one object); a zero-transparency object stops at its first.
__device__ __forceinline__ uint32_t wfp_object_shadow(const DS& S, int o, V3 p, V3 dir, double dist, const CullR& cr) {
  cptr<RtObject> O = &S.objects[o];
  const bool fin = wave_finite(p, dir);
  const bool cf_ok = RT_CONST_FILTER && const_filter_range(p, dir);
  const CullT tmax = RT_CULL_TMAX(dist);
  const bool zero = O->transparency == 0.0;
  uint32_t cnt = 0;
  SphereShare shr = {0.0, 0.0, 0.0};
  const int lb = O->leaf_begin, le = lb + O->leaf_count;
  for (int l = lb; l < le; ++l) {
    cptr<RtLeaf> L = &S.leaves[l];
    if (O->leaf_cull) {
      if (L->cull == RT_CULL_ALWAYS) continue;
      if (L->cull == RT_CULL_BOX && !RT_BOX_MAY_HIT(L, blo, bhi, cr, tmax)) continue;
    }
    double t0 = 0.0, t1 = 0.0;
    const int n = leaf_candidates<true>(L, p, dir, fin, &t0, &t1, RT_SPHERE_SHARE ? &shr : nullptr);
    const bool filtered = L->prog_end != L->prog_begin && !(cf_ok && L->filter_const);
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
    camera_ray_px(S, x, y, ro, rd);
    return true;
  }
  *ro = {lv.ox[j], lv.oy[j], lv.oz[j]};
  *rd = {lv.dx[j], lv.dy[j], lv.dz[j]};
  return true;
}

// One wave per 64 rays of level d (in key order).  SHADOW = false: every object whose box the ray
// meets; true: per light, every object whose box the shadow segment meets (objects of transparency 1
// skipped, as shadow_transparency does).
// Each lane walks its own path through the hierarchy (one 32-byte RtTravC record per step, which
// carries the object's box and flags): a wave-uniform walk visits the union of its 64 rays' paths,
// measured 4-20 % slower here (profiles/r03m_pairs_fractal_timing.txt).
// A step's record load is the walk's latency: one dependent per-lane load per node, ~100 of them
// per deep ray on fractal.scene -- the deep levels' dispatches last 45-90 us with a few hundred
// waves because each wave is that chain (SQ_WAVE_CYCLES counts quad-cycles: the round-3 "8-15 k
// cycles" per wave are 32-60 k, 15-30 us).  LDS_TRAV: the workgroup (WG_WAVES waves) first copies
// the hierarchy into LDS and the walks read it there.  Loading the next record beside the box test
// (the pre-order successor, the next step unless a group misses) measured 9 % slower on the fractal
// frame (6.02 -> 6.58 ms, profiles/r07q_fractal.txt): kept out.
#ifndef RT_WFP_CAND_WAVES_N
#define RT_WFP_CAND_WAVES_N 4
#endif
constexpr int RT_WFP_CAND_WAVES = RT_WFP_CAND_WAVES_N;
constexpr uint32_t RT_WFP_LDS_TRAV_MAX = 1280;    // nodes (40 KB of RtTravC) staged at most; larger: global loads
#ifndef RT_WFP_MAX_RANGES_LOG2
#define RT_WFP_MAX_RANGES_LOG2 2                     // at most 4 hierarchy ranges per ray (below)
#endif
#ifndef RT_WFP_CAND_COUNTS
#define RT_WFP_CAND_COUNTS 1                         // the candidate kernels count their pairs for the sorts
#endif
#ifndef RT_WFP_HITSORT_MAX_D
#define RT_WFP_HITSORT_MAX_D 1000                    // levels from this depth on skip the hit-point sort
#endif
#ifndef RT_WFP_RANGE_PASSES
#define RT_WFP_RANGE_PASSES 8                        // ... while the items fill the grid at most 8 times (4: +0.8 %)
#endif
#ifndef RT_WFP_NEAR_RANGES_LOG2
#define RT_WFP_NEAR_RANGES_LOG2 1                    // the nearest pass's walks: at most 2 ranges (8 measured slower)
#endif
// n_dev != nullptr (device-driven levels): the level's ray count is min(*n_dev, A.cap), read here; the
// grid is then a fixed number of workgroups that take the level's rays grid-stride, 64 x WG_WAVES at a
// time (the hierarchy staged in LDS once per workgroup).
template <bool SHADOW, bool LDS_TRAV>
__global__ __launch_bounds__(64 * RT_WFP_CAND_WAVES) void wfp_cand_kernel(RtDevScene S, WfArena A, WfPairs P, int d,
                                                                          uint32_t n, const uint32_t* n_dev,
                                                                          int y_first, int band_rows, int band_pitch,
                                                                          int n_rows, uint32_t* __restrict__ hcnt) {
  constexpr int WW = LDS_TRAV ? RT_WFP_CAND_WAVES : 1;
  __shared__ uint32_t sk_all[WW][RT_WFP_BUF], sv_all[WW][RT_WFP_BUF];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_trav[];
  // hcnt != nullptr: the pairs' histogram by object for the bucket sort (its histogram launch skipped),
  // counted in LDS (after the staged hierarchy) and added to hcnt once per workgroup
  uint32_t* const s_hist = (uint32_t*)(s_trav + (LDS_TRAV ? (size_t)S.n_trav * sizeof(RtTravC) : 0));
  const int lane = threadIdx.x & 63, wv = (int)(threadIdx.x >> 6);
  uint32_t* sk = sk_all[LDS_TRAV ? wv : 0];
  uint32_t* sv = sv_all[LDS_TRAV ? wv : 0];
  if (n_dev) n = min(*n_dev, A.cap);
  // Hierarchy ranges: a small level's rays are too few to fill the grid, and its time is the longest
  // walk of one lane (~100-600 dependent node steps).  There the node array is cut into K equal
  // contiguous ranges and a lane walks one (ray, range) item: the walk from a range's first node
  // to its end with the same steps (skip pointers only jump forward; a group that misses covers only
  // nodes the ray misses too, as its box holds its objects' boxes).  Ancestors outside the range go
  // untested, so an item may emit pairs the whole walk culls: a superset, which the evaluations
  // resolve exactly.  K: a power of two, at most 2^RT_WFP_MAX_RANGES_LOG2, n x K within RT_WFP_RANGE_PASSES grids.
  const uint32_t nthreads = gridDim.x * (64u * WW);
  uint32_t lk = 0;
  while (lk < (SHADOW ? RT_WFP_MAX_RANGES_LOG2 : RT_WFP_NEAR_RANGES_LOG2) &&
         ((uint64_t)n << (lk + 1)) <= (uint64_t)nthreads * RT_WFP_RANGE_PASSES)
    ++lk;
  const uint32_t items = n << lk;
  if (blockIdx.x * (64u * WW) >= items) return;              // no ray for this workgroup: no staging either
  if (hcnt)
    for (uint32_t b = threadIdx.x; b < (uint32_t)S.n_objects; b += blockDim.x) s_hist[b] = 0;
  if constexpr (LDS_TRAV) {                                   // the hierarchy into LDS, once per workgroup
    const uint4* g = (const uint4*)S.trav_c;
    uint4* l = (uint4*)s_trav;
    for (uint32_t q = threadIdx.x; q < (uint32_t)S.n_trav * (sizeof(RtTravC) / 16); q += blockDim.x) l[q] = g[q];
  }
  if (LDS_TRAV || hcnt) __syncthreads();
  const WfLevel lv = wf_level(A, d);
  const DS D = make_ds(S);
  uint32_t nb = 0;                                           // wave-uniform fill of the LDS buffer
  auto wave_sync = []() {                                    // the wave's own buffer: a wave-level barrier
    if constexpr (LDS_TRAV) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    } else {
      __syncthreads();
    }
  };
  auto flush = [&]() {
    wave_sync();
    uint32_t base = 0;
    if (lane == 0) {
      base = atomicAdd(P.count + (SHADOW ? 1 : 0), nb);
      // a 32-bit count past 2^31 (the arena's limit) is about to wrap: flag the level as failed (the
      // writes below stay inside the arena; the host reports the overflow instead of using the pairs)
      if (base >= 0x80000000u) atomicOr(P.count + 2, 1u);
    }
    base = (uint32_t)__shfl((int)base, 0);
    // the histogram counts the pairs the list holds (a level that overflows it is rendered again, but
    // its sort must still see counts that match the stored keys: no unwritten slot is read)
    for (uint32_t q = (uint32_t)lane; q < nb; q += 64)
      if (base + q < P.cap) {
        P.key[base + q] = sk[q];
        P.val[base + q] = sv[q];
        if (hcnt) atomicAdd(&s_hist[sk[q]], 1u);
      }
    wave_sync();
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
  auto walk = [&](bool act0, V3 o, V3 dir, double tmax, uint32_t id, int t0, int nt) {   // nodes [t0, nt)
    const CullRayF cr = cull_ray_f(o, dir);
    const float tm = (float)tmax;
    const RtTravC* __restrict__ TR = LDS_TRAV ? (const RtTravC*)(const void*)s_trav : S.trav_c;
    int t = act0 ? t0 : nt;
    while (__ballot(t < nt)) {
      bool h = false;
      int ob = 0;
      if (t < nt) {
        const RtTravC T = TR[t];
        const bool in = fbox_may_hit(T.lo, T.hi, cr, tm);
        const int cull = (int)((T.skip_flags >> 28) & 3u);
        if (T.obj < 0) {
          t = in ? t + 1 : (int)(T.skip_flags & 0x0fffffffu);
        } else {
          ++t;
          ob = T.obj;
          h = cull != RT_CULL_ALWAYS && !(SHADOW && (T.skip_flags >> 30)) && (cull != RT_CULL_BOX || in);
        }
      }
      emit(h, (uint32_t)ob, id);
    }
  };
  for (uint32_t base = blockIdx.x * (64u * WW); base < items; base += nthreads) {   // wave-uniform
    const uint32_t q = base + threadIdx.x, i = q >> lk, rg = q & ((1u << lk) - 1u);
    // this item's range of the node array (the whole array when K = 1)
    const int t0 = (int)(((uint32_t)S.n_trav * rg) >> lk), t1 = (int)(((uint32_t)S.n_trav * (rg + 1u)) >> lk);
    bool live = q < items;
    uint32_t j = i;
    V3 ro = {0.0, 0.0, 0.0}, rd = {0.0, 0.0, 0.0};
    if (live) {
      j = SHADOW ? P.hperm[i] : (d > 0 && A.perm) ? A.perm[i] : i;
      if (!SHADOW) live = wf_get_ray(S, lv, d, j, y_first, band_rows, band_pitch, n_rows, &ro, &rd);
    }
    if constexpr (!SHADOW) {
      if (q < items && rg == 0) { P.tmin[j] = RT_WFP_NONE; P.omin[j] = 0x7fffffff; }   // slots outside the frame too
      // A bound on the nearest hit: the object whose hit spawned the ray, evaluated first (a ray that
      // refracted into or reflects inside a closed shape meets it again).  The walk then tests boxes
      // against [0, cull_tmax(bound)] only -- conservative, as nearest_hit's running best is; the
      // parent's own pair is still emitted by the walk (its box contains the bound's point).
      double bound = INFINITY;
      if (d > 0) {
        const int32_t par = live ? lv.par[j] : -1;
        const CullR cr = RT_CULL_RAY(ro, rd);
        uint64_t todo = __ballot(live && par >= 0);
        while (todo) {                     // the children of one shading wave: mostly one parent
          const int pu = __builtin_amdgcn_readlane(par, (int)__builtin_ctzll(todo));
          const uint64_t mine = __ballot(live && par == pu);
          todo &= ~mine;
          if ((mine >> lane) & 1) bound = wfp_object_nearest(D, pu, ro, rd, cr);
        }
      }
      walk(live, ro, rd, bound < INFINITY ? cull_tmax(bound) : INFINITY, j, t0, t1);
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
          if (rg == 0) {
            P.kcnt[s] = 0;
            P.opq[s] = 0;
          }
        }
        walk(hit, p, sdir, tmax, s, t0, t1);
      }
    }
  }
  flush();
  if (hcnt) {                                                // every wave of the workgroup is done
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < (uint32_t)S.n_objects; b += blockDim.x)
      if (s_hist[b]) atomicAdd(&hcnt[b], s_hist[b]);
  }
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
    const CullR cr = RT_CULL_RAY(ro, rd);
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
                                                          const uint32_t* n_dev, int y_first, int band_rows,
                                                          int band_pitch, int n_rows, int cbits) {
  if (n_dev) n = min(*n_dev, A.cap);
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
    const CullR cr = RT_CULL_RAY(p, sdir);
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
__device__ __forceinline__ void wfp_shade_one(RtDevScene S, WfArena A, WfPairs P, const WfLevel& lv, int d, uint32_t i,
                                              uint32_t n, int lane, int y_first, int band_rows, int band_pitch,
                                              int n_rows, int max_depth) {
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


// The pair counter block P.count (RT_WFP_COUNT words into WfArena::count): [0] / [1] the nearest / shadow
// pairs of the level, [2] a count wrapped; sticky over the launch: [3] the most pairs any level emitted
// beyond the lists' capacity, [4] any wrap; [5 + 2d] / [6 + 2d] (d <= RT_WFP_LOG_LEVELS) the pairs level
// d emitted, for diagnostics.
constexpr int RT_WFP_LOG_LEVELS = (64 - RT_WFP_COUNT - 5) / 2 - 1;
static_assert(RT_WFP_COUNT + 6 + 2 * RT_WFP_LOG_LEVELS < 64, "wavefront counter block: 256 bytes");

// n_dev != nullptr (device-driven levels): the ray count is min(*n_dev, A.cap); the waves take the
// level's rays grid-stride, 64 at a time (wf_append: one ballot + one atomic per wave and chunk).
// The level's last kernel also closes it (every reader of the pair counts and the sort scratch has
// run): thread 0 checks the pair counts against the lists (a level that emitted more pairs than they
// hold computed wrong nearest hits: sticky words the host reads once per launch) and zeroes them, and
// the grid zeroes the three sorts' scratch -- for the next level, with no launches of their own (three
// per level in round 5's first form: 5 us each on the small levels).
template <bool REFR, bool FC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU_WF))) void wfp_shade_kernel(
    RtDevScene S, WfArena A, WfPairs P, int d, uint32_t n, const uint32_t* n_dev, int y_first, int band_rows,
    int band_pitch, int n_rows, int max_depth) {
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && lane == 0) {
    uint32_t* pc = P.count;
    const uint32_t m = max(pc[0], pc[1]);
    if (m > P.cap) atomicMax(pc + 3, m);
    if (pc[2]) atomicOr(pc + 4, 1u);
    if (d <= RT_WFP_LOG_LEVELS) { pc[5 + 2 * d] = pc[0]; pc[6 + 2 * d] = pc[1]; }
    pc[0] = pc[1] = pc[2] = 0;
  }
  for (uint32_t k = blockIdx.x * 64u + (uint32_t)lane; k < 3u * RT_WFP_BIN_WORDS; k += gridDim.x * 64u) P.bins[k] = 0;
  if (n_dev) n = min(*n_dev, A.cap);
  const WfLevel lv = wf_level(A, d);
  for (uint32_t base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u)   // wave-uniform
    wfp_shade_one<REFR, FC>(S, A, P, lv, d, base + (uint32_t)lane, n, lane, y_first, band_rows, band_pitch, n_rows,
                            max_depth);
}

}  // namespace

using namespace rt;

extern "C" hipError_t rt_wf_bucket_sort(const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                                        uint32_t* vals_out, uint32_t n, const uint32_t* n_dev, uint32_t nb, int shift,
                                        uint32_t* cnt, bool zero_cnt, hipStream_t stream, bool counted = false);
#ifdef RT_WF_RADIX_SORT
extern "C" hipError_t rt_wf_sort_pairs(void* d_temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                       const uint32_t* vals_in, uint32_t* vals_out, int n, int end_bit,
                                       hipStream_t stream);
#endif
#define RT_WF_LEVEL_BINS 4096u          // bucket-sort bins of a non-pair level (the key's top 12 bits)

// Pair-path arrays (above, "wavefront pair path"): per ray of a level (R = the larger of
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
    const size_t bytes = al(3 * RT_WFP_BIN_WORDS * 4 + 4 * cap * 4 + cap * 8);
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
  P->key = (uint32_t*)(b + 3 * RT_WFP_BIN_WORDS * 4);
  P->val = P->key + cap;
  P->key_s = P->val + cap;
  P->val_s = P->key_s + cap;
  P->tp = (double*)(P->val_s + cap);
  return RT_OK;
}

// One level of the wavefront path through the pair path: candidate pairs, sort by object, pair
// evaluation and the folds, for the nearest hits and then the shadow rays, then the shading pass.
// Device-driven (round 5): no host synchronisation.  The level's ray count is n (known on the host:
// level 0) or min(A.count[d], cap), read by the kernels themselves (n_dev); the pair counts stay on the
// device too (the sorts and the evaluations read them).  Grids are fixed and the kernels take their
// work grid-stride, so the host launches every level back to back.  A level whose pairs outgrew the
// lists leaves the sticky overflow word (checked by the level's shading kernel); the host reads it once, after the
// whole launch, and renders the launch again with lists of that size (launch_wavefront).
static int wfp_level(rt_ctx* c, hipStream_t st, const WfArena& A, size_t R, int d, uint32_t n_ub, const uint32_t* n_dev,
                     int a0, int a1, int a2, int a3, int max_depth, bool refr, bool fc, bool first) {
  WfPairs P;
  int rc = wfp_arena(c, st, R, A.cap, 0, &P);
  if (rc) return rc;
  P.count = A.count + RT_WFP_COUNT;
  const uint32_t ncu = (uint32_t)c->n_cu;
  auto grid = [&](uint32_t per_wg, uint32_t max_wg) { return dim3(std::max(1u, std::min((n_ub + per_wg - 1) / per_wg, max_wg))); };
  const dim3 b64(64);
  const uint32_t nobj = (uint32_t)c->dev.n_objects;
  uint32_t* bins[3] = {P.bins, P.bins + RT_WFP_BIN_WORDS, P.bins + 2 * RT_WFP_BIN_WORDS};
  // the candidate walks: hierarchies of up to RT_WFP_LDS_TRAV_MAX nodes staged in LDS (4-wave groups)
  const bool lds_trav = (uint32_t)c->dev.n_trav <= RT_WFP_LDS_TRAV_MAX && !diag_env("RT_WFP_GLOBAL_TRAV");
  // the candidate kernels count their pairs by object for the sorts (fused-scan sorts: <= 2048 objects)
  const bool counted = nobj <= RT_WFP_BIN_WORDS / 2 && RT_WFP_CAND_COUNTS;
  const size_t hist_lds = counted ? (size_t)nobj * 4 : 0;
  auto launch_cand = [&](bool shadow) {
    uint32_t* hc = counted ? bins[shadow ? 2 : 0] : nullptr;
    if (lds_trav) {
      // as many workgroups as the CUs hold at once (the LDS-staged hierarchy sets it); they take the
      // level's rays grid-stride and stage the hierarchy once each (round 5's first form launched
      // 16 per CU: on the small levels most of them only staged and found no ray)
      const size_t lds = (size_t)c->dev.n_trav * sizeof(RtTravC) + hist_lds;
      int& occ = c->wfp_occ[shadow ? 1 : 0];                    // queried once per context and LDS size
      if (occ < 1 || c->wfp_occ_lds[shadow ? 1 : 0] != lds) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)(shadow ? wfp_cand_kernel<true, true> : wfp_cand_kernel<false, true>),
                                                         64 * RT_WFP_CAND_WAVES, lds) != hipSuccess || occ < 1)
          occ = 1;
        c->wfp_occ_lds[shadow ? 1 : 0] = lds;
      }
      const dim3 gl = grid(64 * RT_WFP_CAND_WAVES, ncu * (uint32_t)occ), bl(64 * RT_WFP_CAND_WAVES);
      if (shadow) hipLaunchKernelGGL((wfp_cand_kernel<true, true>), gl, bl, lds, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3, hc);
      else hipLaunchKernelGGL((wfp_cand_kernel<false, true>), gl, bl, lds, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3, hc);
    } else if (shadow) {
      hipLaunchKernelGGL((wfp_cand_kernel<true, false>), grid(64, ncu * 64), b64, hist_lds, st, c->dev, A, P, d, n_ub, n_dev,
                         a0, a1, a2, a3, hc);
    } else {
      hipLaunchKernelGGL((wfp_cand_kernel<false, false>), grid(64, ncu * 64), b64, hist_lds, st, c->dev, A, P, d, n_ub, n_dev,
                         a0, a1, a2, a3, hc);
    }
  };
  // grid-stride evaluations: one pass covers ~4 pairs per ray of the level (fractal: ~3), at most 8
  // waves per SIMD
  const dim3 ge(std::max<uint32_t>(ncu, std::min<uint32_t>((uint32_t)(((size_t)n_ub * 4 + 63) / 64), ncu * 32u)));
  // the pair counters start at zero with the launch's counter block; the sorts' scratch is zeroed here
  // for the launch's first pair level, by each level's shading kernel for the next
  if (first) RT_HIP(hipMemsetAsync(P.bins, 0, 3 * RT_WFP_BIN_WORDS * 4, st));
  launch_cand(false);
  RT_HIP(rt_wf_bucket_sort(P.key, P.key_s, P.val, P.val_s, P.cap, P.count, nobj, 0, bins[0], false, st, counted));
  hipLaunchKernelGGL(wfp_near_eval_kernel, ge, b64, 0, st, c->dev, A, P, d, a0, a1, a2, a3);
  hipLaunchKernelGGL(wfp_near_tie_kernel, dim3(std::min<uint32_t>((P.cap + 255) / 256, 4096)), dim3(256), 0, st, P);
  // the hit points and their order for the shadow and shading passes: at most 2048 buckets of
  // (hit object, coarse hit-point cell), unordered within a bucket (a 16^3-cell-only key and the
  // full 27-bit radix sort measured slower: profiles/r03o_sort_ab.txt, r03w_*)
  int cbits = 0;
  while (cbits < 12 && ((nobj + 1u) << (cbits + 1)) <= RT_WFP_BIN_WORDS / 2) ++cbits;   // the fused-scan sort's bins
  // (the hit-key kernel counting its keys for this sort, over contiguous 4096-ray chunks, measured
  // slower: 5.63 vs 5.50 ms, profiles/r08a_fractal.txt)
  hipLaunchKernelGGL(wfp_hit_key_kernel, grid(256, ncu * 8), dim3(256), 0, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3,
                     cbits);
  if (d < RT_WFP_HITSORT_MAX_D)
    RT_HIP(rt_wf_bucket_sort(P.hkey, P.hkey_s, P.hval, P.hperm, n_ub, n_dev, (nobj + 1u) << cbits, 0, bins[1], false, st));
  else
    P.hperm = P.hval;                     // the level's own order (hval[i] = the i-th ray's slot)
  launch_cand(true);
  RT_HIP(rt_wf_bucket_sort(P.key, P.key_s, P.val, P.val_s, P.cap, P.count + 1, nobj, 0, bins[2], false, st, counted));
  hipLaunchKernelGGL(wfp_shadow_eval_kernel, ge, b64, 0, st, c->dev, P);
  const dim3 gs = grid(64, ncu * 32);
  if (refr && fc) hipLaunchKernelGGL((wfp_shade_kernel<true, true>), gs, b64, 0, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3, max_depth);
  else if (refr) hipLaunchKernelGGL((wfp_shade_kernel<true, false>), gs, b64, 0, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3, max_depth);
  else if (fc) hipLaunchKernelGGL((wfp_shade_kernel<false, true>), gs, b64, 0, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3, max_depth);
  else hipLaunchKernelGGL((wfp_shade_kernel<false, false>), gs, b64, 0, st, c->dev, A, P, d, n_ub, n_dev, a0, a1, a2, a3, max_depth);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

// The wavefront path (wf_*_kernel): level 0 (the pixel slots), then each level the previous one
// appended to, sorted by coherence key; then the folds, deepest level first; then the overflow
// fix-up.  The host reads every level's ray count (one stream synchronisation per level) to launch
// exactly one wave per 64 rays and to stop at the first empty level.
int rt::launch_wavefront(rt_ctx* c, hipStream_t st, int a0, int a1, int a2, int a3, int max_depth, uint8_t* target,
                            size_t tstride, bool f64, int rgbi, size_t n_tiles, int retry) {
  const size_t slots = n_tiles * 64, cap = std::max<size_t>(64, (slots * (size_t)c->wf_cap_pct / 100 + 63) & ~(size_t)63);
  if (cap > 0x7fffffffull || slots > 0x7fffffffull) return fail(RT_ERR_UNSUPPORTED, "wavefront launch of %zu pixel slots too large", slots);
  // the non-pair levels' coherence order: the in-tree bucket sort on the key's top 12 bits (direction
  // octant + the 8^3-cell Morton prefix); only the processing order depends on it, never a value
  // (diagnostic builds with RT_WF_RADIX_SORT: the full 30-bit rocPRIM radix sort it replaced)
#ifdef RT_WF_RADIX_SORT
  size_t sort_bytes = 0;
  RT_HIP(rt_wf_sort_pairs(nullptr, &sort_bytes, nullptr, nullptr, nullptr, nullptr, (int)cap, 30, st));
#else
  const size_t sort_bytes = RT_WF_LEVEL_BINS * 4;
#endif
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
  // the pair path's shadow-ray ids (slot * n_lights + light) are 32-bit: launches whose ids would not
  // fit keep the wave walk (its counts are checked against 2^31 on the device, wfp_cand_kernel)
  const bool pairs = c->wf_pairs > 0 && c->dev.shadow_pow != 0 && c->dev.n_objects > 0 && c->dev.n_objects < 4096 &&
                     (uint64_t)std::max(slots, cap) * (uint64_t)std::max(1, c->dev.n_lights) < (1ull << 32);
  auto pairs_level = [&](int d) { return pairs && (d > 0 || c->wf_pairs == 2); };
  // n_level[d]: the level's ray count when the host knows it (level 0, and levels the wave walk traced,
  // whose count it reads); known[d] = false: a device-driven pair level (its kernels read A.count[d])
  uint32_t n_level[RT_MAX_DEPTH_CAP + 2] = {0};
  bool known[RT_MAX_DEPTH_CAP + 2] = {false};
  n_level[0] = (uint32_t)slots;
  known[0] = true;
  bool any_pairs = false;
  int last = 0;
  for (int d = 0; d <= max_depth; ++d) {
    if (!known[d] && !pairs_level(d)) {                      // the wave walk needs the count: read it
      uint32_t cnt = 0;
      RT_HIP(hipMemcpyAsync(&cnt, A.count + d, 4, hipMemcpyDeviceToHost, st));
      RT_HIP(hipStreamSynchronize(st));
      n_level[d] = std::min<uint32_t>(cnt, (uint32_t)cap);
      known[d] = true;
    }
    if (known[d] && n_level[d] == 0) break;
    const uint32_t n = n_level[d];
    last = d;
    A.perm = nullptr;
    if (pairs_level(d)) {
      // the pair path reads a level in slot order: its candidate walks are per lane and its evaluations
      // run in object order (a key sort measured 0.3-0.6 ms per fractal frame slower, profiles/r03o_sort_ab.txt)
      int rc = wfp_level(c, st, A, std::max(slots, cap), d, known[d] ? n : (uint32_t)cap, known[d] ? nullptr : A.count + d,
                         a0, a1, a2, a3, max_depth, refr, fc, !any_pairs);
      if (rc) return rc;
      any_pairs = true;
      continue;                                              // level d + 1: device-driven
    }
    if (d > 0) {                                             // this level's slots in key order
      const WfLevel L = wf_level(A, d);                      // host-side pointer arithmetic only
#ifdef RT_WF_RADIX_SORT
      size_t tb = sort_bytes;
      RT_HIP(rt_wf_sort_pairs(tmp, &tb, L.key, kout, L.val, perm, (int)n, 30, st));
#else
      RT_HIP(rt_wf_bucket_sort(L.key, kout, L.val, perm, n, nullptr, RT_WF_LEVEL_BINS, 30 - 12, (uint32_t*)tmp, true, st));
#endif
      A.perm = perm;
    }
    const dim3 g((n + 63) / 64);
    if (refr && fc) hipLaunchKernelGGL((wf_trace_kernel<true, true>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    else if (refr) hipLaunchKernelGGL((wf_trace_kernel<true, false>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    else if (fc) hipLaunchKernelGGL((wf_trace_kernel<false, true>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    else hipLaunchKernelGGL((wf_trace_kernel<false, false>), g, dim3(64), 0, st, c->dev, A, d, n, a0, a1, a2, a3, max_depth);
    RT_HIP(hipGetLastError());
  }
  // the folds, deepest level first, RT_WF_FOLD_SPAN levels per launch; the deepest level's rays have no
  // children (their colour is their hit record) unless it is level 0, which writes the pixels
  const dim3 bf(256);
  for (int top = last > 0 ? last - 1 : 0; top >= 0;) {
    const int d = std::max(0, top - RT_WF_FOLD_SPAN + 1), span = top - d + 1;
    const uint32_t n = known[d] ? n_level[d] : (uint32_t)cap;
    const uint32_t* nd = known[d] ? nullptr : A.count + d;
    const dim3 gf(std::max(1u, std::min<uint32_t>((n + 255) / 256, (uint32_t)c->n_cu * 8u)));
#define RT_WF_FOLD(SP)                                                                                                  \
  if (f64 && fc) hipLaunchKernelGGL((wf_fold_kernel<SP, true, true>), gf, bf, 0, st, c->dev, A, d, n, nd, a0, a1, a2, a3, target, tstride, rgbi); \
  else if (f64) hipLaunchKernelGGL((wf_fold_kernel<SP, true, false>), gf, bf, 0, st, c->dev, A, d, n, nd, a0, a1, a2, a3, target, tstride, rgbi); \
  else if (fc) hipLaunchKernelGGL((wf_fold_kernel<SP, false, true>), gf, bf, 0, st, c->dev, A, d, n, nd, a0, a1, a2, a3, target, tstride, rgbi); \
  else hipLaunchKernelGGL((wf_fold_kernel<SP, false, false>), gf, bf, 0, st, c->dev, A, d, n, nd, a0, a1, a2, a3, target, tstride, rgbi);
    if (span >= 3) { RT_WF_FOLD(3) }
    else if (span == 2) { RT_WF_FOLD(2) }
    else { RT_WF_FOLD(1) }
#undef RT_WF_FOLD
    top = d - 1;
  }
  const dim3 gx((unsigned)c->n_cu * 4u);
#define RT_WF_FIX(R, F, FCv) hipLaunchKernelGGL((wf_fixup_kernel<R, F, FCv>), gx, dim3(64), 0, st, c->dev, A, a0, a1, a2, a3, max_depth, target, tstride, rgbi)
  if (refr && f64) { if (fc) RT_WF_FIX(true, true, true); else RT_WF_FIX(true, true, false); }
  else if (refr) { if (fc) RT_WF_FIX(true, false, true); else RT_WF_FIX(true, false, false); }
  else if (f64) { if (fc) RT_WF_FIX(false, true, true); else RT_WF_FIX(false, true, false); }
  else { if (fc) RT_WF_FIX(false, false, true); else RT_WF_FIX(false, false, false); }
#undef RT_WF_FIX
  RT_HIP(hipGetLastError());
  if (any_pairs) {
    // the device-driven pair levels' sticky words: ONE host synchronisation per launch (round 4: one per
    // level).  A level whose pairs outgrew the lists computed wrong hits: grow them to what it needed and
    // render the launch again (its levels recomputed from the camera rays; the tests force this path)
    uint32_t ov[2] = {0, 0};
    RT_HIP(hipMemcpyAsync(ov, A.count + RT_WFP_COUNT + 3, sizeof ov, hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
    static const bool wf_debug = diag_env("RT_WF_DEBUG");
    if (wf_debug) {                       // per level: rays, nearest pairs, shadow pairs
      uint32_t cb[64];
      RT_HIP(hipMemcpy(cb, A.count, sizeof cb, hipMemcpyDeviceToHost));
      fprintf(stderr, "wavefront levels (rays / nearest pairs / shadow pairs):");
      for (int d = 0; d <= last && d <= RT_WFP_LOG_LEVELS; ++d)
        fprintf(stderr, " %d: %u / %u / %u;", d, d == 0 ? (uint32_t)slots : cb[d], cb[RT_WFP_COUNT + 5 + 2 * d],
                cb[RT_WFP_COUNT + 6 + 2 * d]);
      fprintf(stderr, "\n");
    }
    if (ov[1]) return fail(RT_ERR_UNSUPPORTED, "wavefront pair count passed 2^31");
    if (ov[0]) {
      if (retry > 2) return fail(RT_ERR_DEVICE, "wavefront pair lists still overflow after %d resizes", retry);
      WfPairs P;
      int rc = wfp_arena(c, st, std::max(slots, cap), cap, (size_t)ov[0], &P);   // grows (synchronises)
      if (rc) return rc;
      return launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles, retry + 1);
    }
  }
  return RT_OK;
}

