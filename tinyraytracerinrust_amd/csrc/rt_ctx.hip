// rt_ctx.hip -- the device context of the C ABI (include/rt_abi.h): device discovery, context
// create / free, scene upload (rt::flatten -> one HBM blob, rt_blob.h), options, own-queue streams.
// Host code only; the kernels and their launches live in k_rows.hip, k_wavefront.hip, k_views.hip.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>

#include "rt_ctx.h"

namespace rt {

bool diag_env(const char* name) {
#ifdef RT_DIAG_ENV
  return getenv(name) != nullptr;
#else
  (void)name;
  return false;
#endif
}

void drop_order(rt_ctx::OrderSlot& s) {
  if (s.d_order) (void)hipFree(s.d_order);     // hipFree waits for work that may still read it
  if (s.d_cost) (void)hipFree(s.d_cost);
  s = rt_ctx::OrderSlot();
}
void drop_orders(rt_ctx* c) {
  for (auto& s : c->order) drop_order(s);
}

int ensure_scratch(rt_ctx* c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return RT_OK;
  if (c->scratch) (void)hipFree(c->scratch);
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  RT_HIP(hipMalloc(&c->scratch, bytes));
  c->scratch_bytes = bytes;
  return RT_OK;
}

// The completion event of stream st for c (created on first use; with more than 16 streams the
// least recently added one's launches are waited for and its event reused).  Row launches BIND it to
// the kernel dispatch itself (hipExtLaunchKernel's stop event: no marker packet of its own); a
// separate hipEventRecord after every launch cost the stream 2.5-3.6 us per launch
// (profiles/r07d_marks_ab.txt: the 1080p sphere 0.0189 -> 0.0218 ms per frame).
int mark_event(rt_ctx* c, hipStream_t st, hipEvent_t* ev) {
  for (auto& m : c->marks)
    if (m.s == st) {
      *ev = m.ev;
      return RT_OK;
    }
  rt_ctx::Mark m{st, nullptr};
  if (c->marks.size() >= 16) {
    m.ev = c->marks.front().ev;
    RT_HIP(hipEventSynchronize(m.ev));
    c->marks.erase(c->marks.begin());
  } else {
    RT_HIP(hipEventCreateWithFlags(&m.ev, hipEventDisableTiming));
  }
  c->marks.push_back(m);
  *ev = m.ev;
  return RT_OK;
}

int mark_launch(rt_ctx* c, hipStream_t st) {
#ifdef RT_DIAG_NO_MARKS
  return RT_OK;                       // diagnostic builds only: the marks' cost (A/B)
#endif
  hipEvent_t ev = nullptr;
  RT_TRY(mark_event(c, st, &ev));
  RT_HIP(hipEventRecord(ev, st));
  return RT_OK;
}

int wait_launches(rt_ctx* c) {
  for (auto& m : c->marks) RT_HIP(hipEventSynchronize(m.ev));
  return RT_OK;
}

bool is_device_ptr(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

}  // namespace rt

using rt::drop_orders;

template <typename T>
static size_t put(std::vector<uint8_t>& blob, const std::vector<T>& v) {
  size_t off = (blob.size() + 255) & ~(size_t)255;
  blob.resize(off + v.size() * sizeof(T) + 16);
  if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
  return off;
}

extern "C" {

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
  std::vector<RtTravC> travc, stravc;
  for (const auto* src : {&f.trav, &f.strav}) {
    std::vector<RtTravC>& dst = src == &f.trav ? travc : stravc;
    dst.resize(src->size());
    for (size_t i = 0; i < src->size(); ++i) {
      const RtTrav& t = (*src)[i];
      if ((uint32_t)t.skip >= (1u << 28)) return fail(RT_ERR_UNSUPPORTED, "object hierarchy of more than 2^28 nodes");
      for (int k = 0; k < 3; ++k) { dst[i].lo[k] = t.fblo[k]; dst[i].hi[k] = t.fbhi[k]; }
      dst[i].obj = t.obj;
      dst[i].skip_flags = (uint32_t)t.skip | (uint32_t)t.cull << 28 | (uint32_t)(t.shadow_skip ? 1 : 0) << 30;
    }
  }
  const size_t o_travc = put(blob, travc), o_stravc = put(blob, stravc);
  size_t o_prog = put(blob, f.prog), o_lights = put(blob, f.lights), o_tex = put(blob, f.textures);
  size_t o_texels = put(blob, f.texels);
  // camera_ray's terms of the integer pixels (rt_device.h camera_ray_px): the same expressions in the
  // same order, IEEE double on the host (-ffp-contract=off as the device), so a table entry is the
  // value the device would compute
  std::vector<double> csx((size_t)std::max(0, f.width)), csy((size_t)std::max(0, f.height));
  for (size_t x = 0; x < csx.size(); ++x) csx[x] = (((double)x / f.cam.width) - 0.5) * f.cam.aspect;
  for (size_t y = 0; y < csy.size(); ++y) csy[y] = (f.cam.height - 1.0 - (double)y) / f.cam.height - 0.5;
  size_t o_csx = put(blob, csx), o_csy = put(blob, csy);
  RT_HIP(hipSetDevice(c->device));
  RT_TRY(rt::wait_launches(c));       // launches in flight read the blob and may run the specialised modules
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
  d.trav_c = (const RtTravC*)(b + o_travc);
  d.strav_c = (const RtTravC*)(b + o_stravc);
  d.n_strav = (int32_t)f.strav.size();
  d.nodes = (const RtNode*)(b + o_nodes);
  d.leaves = (const RtLeaf*)(b + o_leaves);
  d.prog = (const RtProg*)(b + o_prog);
  d.lights = (const RtLight*)(b + o_lights);
  d.textures = (const RtTexture*)(b + o_tex);
  d.texels = b + o_texels;
  d.cam_sx = (const double*)(b + o_csx);
  d.cam_sy = (const double*)(b + o_csy);
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
  // Tile costs belong to the previous scene -- unless the new one has its structure (the same scene
  // rebuilt, or the next frame of an animation: a host shaped like the reference's GUI rebuilds and
  // uploads the scene every frame, debug_window.rs:53-68, gui.rs:78-89).  Then its orders stay: any
  // tile order renders the same pixels, the old one is near the new costs, and the first launch after
  // the upload takes an ordered (non-calibrating) kernel -- the specialised one, whose programs have no
  // calibration variant at the default level (a calibrating launch would run the generic kernels).
  if (!(c->spec_flat && rt::same_structure_flat(*c->spec_flat, f))) drop_orders(c);
  // the scene-specialised programs (spec.hip): requested from the compile pool, loaded by the first
  // launch after they are ready; the generic kernels render until then.  Only the flags are computed
  // here -- the program text (and a family lookup) only when the option is on and the scene fits.
  rt::spec_drop(c);                   // the previous scene's modules (the hipFree above waited for the device)
  c->spec_flat = std::make_shared<rt::FlatScene>(std::move(f));
  c->spec_flat->texels.clear();
  c->spec_flat->texels.shrink_to_fit();
  rt::spec_flags(*c->spec_flat, c);
  rt::spec_prepare(c);
  return RT_OK;
}

int rt_ctx_kernel_info(rt_ctx* c, char* buf, size_t cap) {
  if (!c || !buf || cap == 0) return fail(RT_ERR_INVALID, "null argument");
  std::string s;
  char b[1024];
  if (c->spec_mod) {
    snprintf(b, sizeof b, "scene-specialised (hipRTC %016llx, %s%s, compiled in %.0f ms%s by %s; %s; loaded %.0f ms after "
             "the request)", (unsigned long long)c->spec_hash,
             c->spec_mode == RT_MODE_REFL ? "reflection" : c->spec_mode == RT_MODE_CHAIN ? "chain" : "tree",
             c->spec_family ? (", family of " + std::to_string(c->spec_family) + " scenes").c_str() : "",
             c->spec_compile_ms, c->spec_note.c_str(), rt::spec_compiler(), c->spec_res.c_str(), c->spec_ready_ms);
    s = b;
  } else if (c->spec_on && c->uploaded && !c->spec_fits) {
    snprintf(b, sizeof b, "generic (librt_mi355x.so; scene too large to specialise: > %d objects or > %d leaves)",
             RT_SPEC_MAX_OBJECTS, RT_SPEC_MAX_LEAVES);
    s = b;
  } else if (c->spec_on && c->uploaded && !c->spec_jobs.empty()) {
    s = "generic (librt_mi355x.so; the scene-specialised program is compiling in the background)";
  } else if (c->spec_on && c->uploaded && !c->spec_error.empty()) {
    s = "generic (librt_mi355x.so; specialisation failed: " + c->spec_error + ")";
  } else {
    s = "generic (librt_mi355x.so)";
  }
  s += std::string("; last launch: ") + c->last_kernel;
  snprintf(buf, cap, "%s", s.c_str());
  return RT_OK;
}

int rt_ctx_spec_wait(rt_ctx* c, int32_t timeout_ms) {
  if (!c) return fail(RT_ERR_INVALID, "null context");
  RT_HIP(hipSetDevice(c->device));
  const int rc = rt::spec_wait(c, (double)timeout_ms);
  if (rc == RT_PENDING) return RT_PENDING;
  if (!c->spec_error.empty()) return fail(RT_ERR_UNSUPPORTED, "%s", c->spec_error.c_str());
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
  if (option == RT_OPT_SPECIALIZE) {
    if (value < 0 || value > 2) return fail(RT_ERR_INVALID, "RT_OPT_SPECIALIZE value %d", value);
    const bool retry = value == c->spec_on && !c->spec_error.empty();   // the same value again: compile again
    if (value == c->spec_on && !retry) return RT_OK;
    RT_HIP(hipSetDevice(c->device));
    int rc = rt::wait_launches(c);              // this context's launches in flight may still run the modules
    if (rc) return rc;
    rt::spec_drop(c);
    c->spec_on = value;
    if (c->uploaded) rt::spec_prepare(c, retry);   // a scene family registered since the upload may hold it
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
  return rt::wait_launches(c);
}

void rt_ctx_free(rt_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  // this context's own launches, through its completion events: not the device (other contexts'
  // work), not a caller's stream (bench.py's frames-in-flight streams are destroyed by now;
  // synchronising a destroyed stream crashed at exit in round 4)
  (void)rt::wait_launches(c);
  for (auto& m : c->marks) (void)hipEventDestroy(m.ev);
  c->marks.clear();
  if (c->d_blob) (void)hipFree(c->d_blob);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->wf) (void)hipFree(c->wf);
  if (c->wfr) (void)hipFree(c->wfr);
  if (c->wfp) (void)hipFree(c->wfp);
  drop_orders(c);
  rt::spec_drop(c);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->tev0) (void)hipEventDestroy(c->tev0);
  if (c->tev1) (void)hipEventDestroy(c->tev1);
  delete c;
}

}  // extern "C"
