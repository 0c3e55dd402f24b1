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

namespace rt { struct SpecJob; }        // spec.hip: one program's compile, shared by the contexts that want it

struct rt_ctx {
  int device = 0;
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
  int wfp_occ[2] = {0, 0};              // candidate kernels (nearest, shadow): workgroups per CU at wfp_occ_lds bytes of LDS
  size_t wfp_occ_lds[2] = {0, 0};
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
  // Scene-specialised row kernels (spec.hip, rt_ctx_set_option(RT_OPT_SPECIALIZE)): hipRTC compiles
  // rt_device.h with this scene's tables as constexpr data, in the background (the library's compile
  // pool); launches take them once they are loaded (spec_poll), the generic kernels until then.
  int spec_on = 1;                      // RT_OPT_SPECIALIZE: 0 off, 1 (default) product launches, 2 every row launch
  std::string spec_src;                 // the program's prelude (spec_source, or a registered family's)
  int spec_mode = 0;                    // RT_MODE_* of the uploaded scene
  bool spec_fc = false;                 // the program's clamp form (RtDevScene::colour_fast)
  bool spec_deferred = false;           // the program also holds the deferred kernels
  bool spec_fits = false;               // small enough to specialise (RT_SPEC_MAX_OBJECTS / _LEAVES)
  hipModule_t spec_mod = nullptr;       // non-null once the kernels are loaded (null: generic kernels)
  hipModule_t spec_mods[12] = {};       // one module per specialised kernel, on this context's device
  hipFunction_t spec_rows[2][2] = {};   // [f64][cal]
  hipFunction_t spec_def[2][2] = {};    // [f64][cal]
  hipFunction_t spec_prim[2][2] = {};   // [f64][cal]: the primary-ray kernel (max_depth 0 launches)
  uint64_t spec_hash = 0;               // FNV-1a of the prelude (kernel info only; caches compare full texts)
  double spec_compile_ms = 0.0;         // the hipRTC time of the loaded programs (0: read from the disk cache)
  int spec_family = 0;                  // > 0: the program of a registered scene family of that many members
  std::shared_ptr<rt::FlatScene> spec_flat;   // the uploaded scene's tables (texels dropped): the program is
                                        // chosen when the option is set (families registered since the upload)
  std::vector<std::shared_ptr<rt::SpecJob>> spec_jobs;   // programs requested, not yet loaded (one per kernel)
  std::string spec_error;               // why the context keeps the generic kernels although spec_on (kernel info)
  std::string spec_note;                // " [process cache]" / " [disk cache]"
  std::string spec_res;                 // the loaded megakernel's resources (kernel info)
  double spec_t0 = 0.0;                 // when the programs were requested (steady clock, ms)
  double spec_ready_ms = 0.0;           // request -> loaded, ms
  // Completion marks: per stream this context launched on, an event recorded after its last launch
  // there.  rt_ctx_synchronize / option changes / rt_ctx_free wait on them -- never on a caller's
  // stream, which may be destroyed by then.
  struct Mark { hipStream_t s; hipEvent_t ev; };
  std::vector<Mark> marks;
  const char* last_kernel = "none";     // what the last row launch ran (rt_ctx_kernel_info)
};

using rt::fail;

#define RT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

#define RT_TRY(call)                                                                   \
  do {                                                                                 \
    const int rc_ = (call);                                                            \
    if (rc_) return rc_;                                                               \
  } while (0)

#ifndef RT_SPEC_MAX_OBJECTS
#define RT_SPEC_MAX_OBJECTS 32
#endif
#ifndef RT_SPEC_MAX_LEAVES
#define RT_SPEC_MAX_LEAVES 48
#endif
#define RT_SPEC_MAX_FAMILIES 16

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
                     size_t tstride, bool f64, int rgbi, size_t n_tiles, int retry = 0);
// Completion marks (rt_ctx.hip): record one after every launch of the context on stream st; wait for all
int mark_event(rt_ctx* c, hipStream_t st, hipEvent_t* ev);   // the event a launch on st binds as its stop event
int mark_launch(rt_ctx* c, hipStream_t st);                  // record it after work enqueued on st (other launches)
int wait_launches(rt_ctx* c);
// spec.hip: the specialised programs of the uploaded scene -- flags (at upload, cheap), the request to the
// compile pool (asynchronous), the load once compiled (at the next launch, or spec_wait), release
void spec_flags(const FlatScene& f, rt_ctx* c);     // the scene's mode, clamp form, size limits
bool same_structure_flat(const FlatScene& a, const FlatScene& b);   // spec.hip: a scene family's structure test
void spec_prepare(rt_ctx* c, bool retry = false);   // request c's programs (spec_on, spec_flat); returns at once
int spec_poll(rt_ctx* c);                           // load them if compiled: RT_OK, or RT_PENDING (spec_error on failure)
int spec_wait(rt_ctx* c, double timeout_ms);        // block (< 0: no limit) then spec_poll
void spec_drop(rt_ctx* c);                          // unload + release (no launch of c may be in flight)
const char* spec_compiler();                        // which hipRTC compiles the programs
}  // namespace rt
