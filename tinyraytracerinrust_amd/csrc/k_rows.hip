// k_rows.hip -- the row kernels (one thread per pixel, one wave per 8x8 tile) and their launches:
// rt_render_rows / _f64 / _row_bands / _row_bands_rgb8 (include/rt_abi.h), i.e. the reference's row
// loop DebugWindow::render_lines (raydebugger/debug_window.rs:74-87) over get_pixel
// (raytracer/raytracer.rs:359-363).  The per-ray code is rt_device.h's.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "rt_device.h"
#include "rt_ctx.h"
#include <hip/hip_ext.h>

namespace {

// The megakernel: trace() per lane (rt_device.h rows_body).  Waves per SIMD per mode: see
// RT_WAVES_MODE.  The first frames of the per-lane stack live in LDS.
template <int MODE, bool F64, bool CAL = false, bool FC = false>
__global__ __launch_bounds__(RT_WG_THREADS) __attribute__((amdgpu_waves_per_eu(RT_WAVES_MODE(MODE)))) void
render_rows_kernel(RtDevScene S, int y_first, int band_rows, int band_pitch, int n_rows, int max_depth,
                   uint8_t* __restrict__ out, size_t stride, const int32_t* __restrict__ order,
                   uint32_t* __restrict__ cost, int rgb) {
  __shared__ double s_frames[rows_lds_doubles<MODE>()];   // frame stack, see trace()
  rows_body<MODE, F64, CAL, FC>(S, y_first, band_rows, band_pitch, n_rows, max_depth, out, stride, order, cost, rgb,
                                (lds_f64*)s_frames);
}

// The deferred-shadow kernel (rt_device.h deferred_body), for launches of few tiles (a multi-GPU
// rank's share) whose time is set by their costliest tiles.  A kernel of its own: the megakernel path
// and this one in ONE kernel measured 3.4x slower than either (profiles/r02g_ab.txt: both paths' code
// hot on one CU at once).
template <bool F64, bool CAL = false, bool FC = false, bool REFR = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU_DEFERRED))) void
render_rows_deferred_kernel(RtDevScene S, int y_first, int band_rows, int band_pitch, int n_rows, int max_depth,
                            uint8_t* __restrict__ out, size_t stride, const int32_t* __restrict__ order,
                            uint32_t* __restrict__ cost, int rgb) {
  __shared__ ShadowWin win;
  deferred_body<F64, CAL, FC, REFR>(S, y_first, band_rows, band_pitch, n_rows, max_depth, out, stride, order, cost, rgb,
                                    &win);
}

}  // namespace

using namespace rt;

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

// Launches with fewer tiles than this are dispatched row-major without a calibration launch: a
// small band (a single row, one rank's sliver) has no tail worth reordering, and calibrating it
// would cost a host synchronisation per new geometry.
#ifndef RT_ORDER_MIN_TILES
#define RT_ORDER_MIN_TILES 2048
#endif

// Primary-ray launches (max_depth 0: one intersection and its shading per pixel, so the frame's
// stores are a large share of the kernel) take an XCD-aware tile order.  The RGBA8 frame's 128-byte
// lines each hold one row of `group` horizontally adjacent 8x8 tiles; cost-sorted, those tiles run at
// different times on different XCDs (workgroups are dealt to the 8 XCDs round-robin: entries e and
// e + 8 share one).  The XCD-aware order keeps the cost sort at the granularity of a line's tiles
// (their costliest first) and places one line's tiles at entries e, e + 8, e + 16, ... of a block of
// 8 x group entries: one XCD renders them back to back.  Measured on every launch
// (profiles/r07n_xcd_order_ab.txt): the sphere 1080p d0 -3 %, globes 1080p d5 -1.2 %, 4K -0.2 %, but
// anim120 1.6 % slower and the partial-line writes do not merge (4K WRITE_SIZE +36 MiB); with plain
// stores as well the sphere gains 9 % but a store-policy branch costs the deeper launches up to 3 %
// (profiles/r08o_xcdp_ab.txt, r08q_cached_ab.txt) -- so the order alone, for max_depth 0 only.
static void xcd_line_order(std::vector<int32_t>& order, const std::vector<uint32_t>& cost, int tiles_x, int group) {
  const size_t n = order.size(), nq = n / (size_t)group, qx = (size_t)(tiles_x / group);
  std::vector<uint32_t> qcost(nq, 0);
  for (size_t t = 0; t < n; ++t) {
    const size_t q = (t / (size_t)tiles_x) * qx + (t % (size_t)tiles_x) / (size_t)group;
    qcost[q] = std::max(qcost[q], cost[t]);
  }
  std::vector<int32_t> qorder(nq);
  for (size_t q = 0; q < nq; ++q) qorder[q] = (int32_t)q;
  std::stable_sort(qorder.begin(), qorder.end(), [&](int32_t x, int32_t y) { return qcost[x] > qcost[y]; });
  size_t e = 0;
  for (size_t g = 0; g < nq; g += 8) {
    const size_t m = std::min<size_t>(8, nq - g);
    for (int j = 0; j < group; ++j)
      for (size_t i = 0; i < m; ++i) {
        const size_t q = (size_t)qorder[g + i];
        order[e++] = (int32_t)((q / qx) * (size_t)tiles_x + (q % qx) * (size_t)group + (size_t)j);
      }
  }
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
  (void)spec_poll(c);                     // the scene-specialised kernels, once their background compile is done
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
    c->last_kernel = "wavefront";
    if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
    c->timed = c->timing;
    RT_TRY(mark_launch(c, st));
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
  const bool chain = refr && c->dev.ray_chains != 0;
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
      RT_HIP(hipMalloc((void**)&slot->d_order, n_tiles * sizeof(int32_t)));
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
  bool deferred;
  if (!eligible || dmode == 0) deferred = false;
  else if (dmode == 1) deferred = true;
  else if (!auto_ok) deferred = false;
  else if (order) deferred = slot->deferred;
  else if (calibrate) deferred = false;                       // calibrate on the megakernel
  else deferred = n_tiles < RT_ORDER_MIN_TILES || (!c->tile_order && n_tiles < RT_DEFERRED_MAX_TILES);
  if (c->timing) RT_HIP(hipEventRecord(c->ev0, st));
  // the row kernels carry the context's completion event for this stream as their stop event
  hipEvent_t mev = nullptr;
#ifndef RT_DIAG_NO_MARKS
  RT_TRY(mark_event(c, st, &mev));
#endif
#define RT_LAUNCH_ROWS(R, F)                                                                                  \
  if (calibrate && fc) hipExtLaunchKernelGGL((render_rows_kernel<R, F, true, true>), grid, block, 0, st, nullptr, mev, 0, \
                                             c->dev, a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);     \
  else if (calibrate) hipExtLaunchKernelGGL((render_rows_kernel<R, F, true, false>), grid, block, 0, st, nullptr, mev, 0, \
                                            c->dev, a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);      \
  else if (fc) hipExtLaunchKernelGGL((render_rows_kernel<R, F, false, true>), grid, block, 0, st, nullptr, mev, 0, c->dev, \
                                     a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);                     \
  else hipExtLaunchKernelGGL((render_rows_kernel<R, F, false, false>), grid, block, 0, st, nullptr, mev, 0, c->dev, a0, a1, \
                             a2, a3, max_depth, target, tstride, order, cost, rgbi);
#define RT_LAUNCH_DEFERRED(F, R)                                                                                \
  if (calibrate && fc) hipExtLaunchKernelGGL((render_rows_deferred_kernel<F, true, true, R>), grid, dim3(64), 0, st,     \
                                             nullptr, mev, 0, c->dev, a0, a1, a2, a3, max_depth, target, tstride, order,  \
                                             cost, rgbi);                                                                 \
  else if (calibrate) hipExtLaunchKernelGGL((render_rows_deferred_kernel<F, true, false, R>), grid, dim3(64), 0, st,     \
                                            nullptr, mev, 0, c->dev, a0, a1, a2, a3, max_depth, target, tstride, order,   \
                                            cost, rgbi);                                                                  \
  else if (fc) hipExtLaunchKernelGGL((render_rows_deferred_kernel<F, false, true, R>), grid, dim3(64), 0, st, nullptr,   \
                                     mev, 0, c->dev, a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);      \
  else hipExtLaunchKernelGGL((render_rows_deferred_kernel<F, false, false, R>), grid, dim3(64), 0, st, nullptr, mev, 0,   \
                             c->dev, a0, a1, a2, a3, max_depth, target, tstride, order, cost, rgbi);
  const bool fc = c->dev.colour_fast != 0 && c->fast_clamp;
  // Ray-tree scenes (a transparent AND reflective object) under RT_KERNEL_AUTO: the first ordered
  // launch of a geometry is timed against one wavefront launch of the same rows, and the faster
  // path takes every later launch (fractal.scene 1080p: 16.4 vs 25.9 ms, profiles/r03d_timing.txt;
  // the small ray-tree scenes of the fuzz suite mostly keep the megakernel).  Same pixels either way.
  const bool tree = refr && !chain;
  if (order && tree && slot->wf_tune == 2) {
    int rc = launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles);
    if (rc) return rc;
    c->last_kernel = "wavefront";
    if (c->timing) RT_HIP(hipEventRecord(c->ev1, st));
    c->timed = c->timing;
    RT_TRY(mark_launch(c, st));
    if (!dev_out) {
      RT_HIP(hipMemcpy2DAsync(out, stride, target, tstride, row_bytes, n_rows, hipMemcpyDeviceToHost, st));
      RT_HIP(hipStreamSynchronize(st));
    }
    return RT_OK;
  }
  const bool tune = order && tree && dmode == -1 && slot->wf_tune == 0;
  if (tune) RT_HIP(hipEventRecord(c->tev0, st));
  const int mode = chain ? RT_MODE_CHAIN : refr ? RT_MODE_TREE : RT_MODE_REFL;
  // the scene-specialised kernel of this launch (spec.hip), when the context holds one that matches
  hipFunction_t sfn = nullptr;
  bool prim = false;
  if (c->spec_mod && mode == c->spec_mode && fc == c->spec_fc) {
    // launches of primary rays only (max_depth 0) take the program's primary-ray kernel (no frame stack,
    // rt_device.h PRIM) unless the deferred kernel was asked for
    prim = max_depth == 0 && dmode != 1 && c->spec_prim[f64 ? 1 : 0][calibrate ? 1 : 0];
    if (prim) deferred = false;
    sfn = prim ? c->spec_prim[f64 ? 1 : 0][calibrate ? 1 : 0]
               : deferred ? c->spec_def[f64 ? 1 : 0][calibrate ? 1 : 0] : c->spec_rows[f64 ? 1 : 0][calibrate ? 1 : 0];
  }
  c->last_kernel = prim ? "primary-ray (specialised)"
                        : deferred ? (sfn ? "deferred (specialised)" : "deferred") : (sfn ? "megakernel (specialised)" : "megakernel");
  if (sfn) {
    void* kargs[] = {&c->dev, (void*)&a0, (void*)&a1, (void*)&a2, (void*)&a3, &max_depth, &target, &tstride,
                     (void*)&order, &cost, (void*)&rgbi};
    // hipExtModuleLaunchKernel takes the global work size in work-items (grid x 64)
    RT_HIP(hipExtModuleLaunchKernel(sfn, grid.x * 64u, 1, 1, 64, 1, 1, 0, st, kargs, nullptr, nullptr, mev, 0));
  }
  else if (deferred && chain && f64) { RT_LAUNCH_DEFERRED(true, true) }
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
    // one untimed wavefront launch first: it allocates (or grows) the wavefront and pair arenas, which
    // the megakernel's timed launch had no counterpart of (a cold first launch could otherwise decide
    // the choice for the geometry)
    int rc = launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles);
    if (rc) return rc;
    RT_HIP(hipEventRecord(c->tev0, st));
    rc = launch_wavefront(c, st, a0, a1, a2, a3, max_depth, target, tstride, f64, rgbi, n_tiles);
    if (rc) return rc;
    RT_HIP(hipEventRecord(c->tev1, st));
    RT_HIP(hipEventSynchronize(c->tev1));
    RT_HIP(hipEventElapsedTime(&wf_ms, c->tev0, c->tev1));
    slot->wf_tune = wf_ms < mega_ms ? 2 : 1;
    static const bool order_debug = diag_env("RT_TILE_ORDER_DEBUG");
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
    // With the scene-specialised megakernel loaded for these launches its costliest tiles finish so
    // much sooner that the deferred kernel no longer pays anywhere: lone 4K rank shares at N = 4 / 8
    // (tail ratios 1.6 / 3.0) 0.109 / 0.098 ms against 0.156 / 0.117 ms deferred, 1080p d5 (ratio 1.6)
    // 0.104 against 0.136 ms (profiles/r06d_kernel_choice.txt): the tail-bound choice is for the
    // generic kernels only.
    const bool spec_mega = c->spec_mod && c->spec_mode == RT_MODE_REFL && c->spec_rows[f64 ? 1 : 0][0] && fc == c->spec_fc;
    if (auto_ok && dmode == -1 && n_tiles < RT_DEFERRED_MAX_TILES && !spec_mega) {
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
      if (split.size() > n_tiles) {                 // more entries than the calibration's table holds
        int32_t* d = nullptr;
        RT_HIP(hipMalloc((void**)&d, split.size() * sizeof(int32_t)));
        (void)hipFree(slot->d_order);
        slot->d_order = d;
      }
      h_order.swap(split);
    }
    const int line_tiles = 128 / (RT_TILE_W * 4);
    if (max_depth == 0 && !f64 && !rgbi && !slot->deferred && tiles_x % line_tiles == 0 && tstride % 128 == 0 &&
        ((uintptr_t)target & 127) == 0)
      xcd_line_order(h_order, h_cost, tiles_x, line_tiles);
    slot->grid = (uint32_t)h_order.size();
    RT_HIP(hipMemcpyAsync(slot->d_order, h_order.data(), h_order.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    RT_HIP(hipStreamSynchronize(st));
    slot->valid = true;
    static const bool order_debug = diag_env("RT_TILE_ORDER_DEBUG");
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

extern "C" {

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

}  // extern "C"
