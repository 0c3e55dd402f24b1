// k_views.hip -- the kernels around the row loop, behind the same C ABI (get_pixel at any point: k_points.hip):
// the ray-debugger recording
// (rt_record_rays; ray_debugger.rs:92-137), the adaptive anti-aliasing pass (rt_antialias;
// antialiaser.rs:87-191), the orthogonal preview views (rt_render_ortho; debug_window.rs:166-227) and
// the multi-GPU frame assembly (rt_assemble_row_bands*; debug_window.rs:147-163).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "rt_device.h"
#include "rt_ctx.h"

namespace {

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

using namespace rt;

extern "C" {

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
  RT_TRY(rt::mark_launch(c, st));
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
  RT_TRY(rt::mark_launch(c, st));
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
  if (refr)
    hipLaunchKernelGGL((record_ray_kernel<true>), dim3(1), dim3(64), 0, st, c->dev, x, y, (int)max_depth, d_rec, d_ord, dev_cap, d_cnt);
  else
    hipLaunchKernelGGL((record_ray_kernel<false>), dim3(1), dim3(64), 0, st, c->dev, x, y, (int)max_depth, d_rec, d_ord, dev_cap, d_cnt);
  RT_HIP(hipGetLastError());
  RT_TRY(rt::mark_launch(c, st));
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

}  // extern "C"
