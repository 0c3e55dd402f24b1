// rt_ctx.h -- the device context behind the C ABI (include/rt_abi.h: rt_ctx_*), shared by the
// host halves of the kernel translation units: rt_ctx.hip (create / upload / options / streams),
// k_rows.hip (the row kernels' launches), k_wavefront.hip, k_views.hip.  Host code only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "rt_blob.h"
#include "scene.h"

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
    int32_t* d_tail = nullptr;        // deferred launches of reflection-only scenes: the costliest tiles, rendered by
    uint32_t n_tail = 0;              //   the tail kernel (G lanes per pixel) on tail_stream, not by the main launch
  };
  static constexpr int RT_ORDER_SLOTS = 8;
  OrderSlot order[RT_ORDER_SLOTS];
  uint64_t use_clock = 0;
  // Scene-specialised row kernels (spec.hip, rt_ctx_set_option(RT_OPT_SPECIALIZE)): hipRTC compiles
  // rt_device.h with this scene's tables as constexpr data; launches take them when they match.
  int spec_on = 0;                      // RT_OPT_SPECIALIZE: 0 off, 1 product launches, 2 every row launch
  std::string spec_src;                 // the program text of the uploaded scene (spec_source)
  int spec_mode = 0;                    // RT_MODE_* of the uploaded scene
  bool spec_fc = false;                 // the program's clamp form (RtDevScene::colour_fast)
  bool spec_deferred = false;           // the program also holds the deferred kernels
  bool spec_fits = false;               // small enough to specialise (RT_SPEC_MAX_OBJECTS / _LEAVES)
  hipModule_t spec_mod = nullptr;       // non-null once the kernels are loaded (null: generic kernels)
  hipModule_t spec_mods[8] = {};        // one module per specialised kernel, on this context's device
  hipFunction_t spec_rows[2][2] = {};   // [f64][cal]
  hipFunction_t spec_def[2][2] = {};    // [f64][cal]
  uint64_t spec_hash = 0;               // FNV-1a of the program text (the code-object cache key)
  double spec_compile_ms = 0.0;         // 0 when the code object came from the process cache
  int spec_family = 0;                  // > 0: the program of a registered scene family of that many members
  std::shared_ptr<rt::FlatScene> spec_flat;   // the uploaded scene's tables (texels dropped): the program is
                                        // re-chosen when the option is set (families registered since)
  const char* last_kernel = "none";     // what the last row launch ran (rt_ctx_kernel_info)
  int tail_tiles = 0;                   // rt_ctx_set_option(RT_OPT_TAIL_TILES): tiles the tail kernel takes (0: none)
  size_t tbl_bytes = 0;                 // the blob's tables [objects, texels): what the tail kernel stages in LDS
  hipStream_t tail_stream = nullptr;    // the tail kernel's stream (a hardware queue of its own), made on first use
  hipEvent_t tail_ev0 = nullptr, tail_ev1 = nullptr;
};

using rt::fail;

#define RT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

#define RT_TAIL_MAX_TABLE_BYTES (48 * 1024)
#define RT_SPEC_MAX_OBJECTS 32
#define RT_SPEC_MAX_LEAVES 48

namespace rt {
// rt_ctx.hip
void drop_order(rt_ctx::OrderSlot& s);         // frees an order table (hipFree waits for its readers)
void drop_orders(rt_ctx* c);
int ensure_scratch(rt_ctx* c, size_t bytes);   // grow-only device scratch for host-pointer launches
bool is_device_ptr(const void* p);
// Diagnostic switches read from the environment exist only in a diagnostic build (make diag
// DIAG=-DRT_DIAG_ENV): RT_TILE_ORDER_DEBUG (rt_ctx.hip / k_rows.hip: tile-cost statistics and the
// kernel each calibration picked, on stderr) and scene.cpp's flattening switches.  The product
// reads no environment variable.
bool diag_env(const char* name);
// k_wavefront.hip: the wavefront path for rows (y_first, band_rows, band_pitch, n_rows) = a0..a3
int launch_wavefront(rt_ctx* c, hipStream_t st, int a0, int a1, int a2, int a3, int max_depth, uint8_t* target,
                     size_t tstride, bool f64, int rgbi, size_t n_tiles);
// k_tail.hip: the tail kernel over n_tail tiles (their indices in d_tail) on stream st
int launch_tail(rt_ctx* c, hipStream_t st, uint32_t n_tail, int a0, int a1, int a2, int a3, int max_depth,
                uint8_t* target, size_t tstride, const int32_t* d_tail, int rgbi, bool fc);
// spec.hip: the specialised program of a flattened scene (at upload), its build (hipRTC, cached per
// process, module loaded on the context's device) and release
void spec_program(const FlatScene& f, rt_ctx* c);   // the scene's mode, clamp form and program text
int spec_build(rt_ctx* c);
void spec_drop(rt_ctx* c);
const char* spec_compiler();                        // which hipRTC compiles the programs
}  // namespace rt
