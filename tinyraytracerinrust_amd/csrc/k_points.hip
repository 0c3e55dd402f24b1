// k_points.hip -- scene-level get_pixel at any (x, y) (rt_render_points_f64, rt_trace_pixel_f64;
// raytracer.rs:359-363), the path the parity tests' chosen points take.  Its own translation unit so
// that its traversals cull with the specialised programs' f32 slab tests (RT_CULL_F32, rt_device.h
// fbox_may_hit) on the same outward-rounded boxes: the edge tests (tests/test_gpu_cull_edges.py,
// test_gpu_texel_boundary.py) aim rays at silhouettes and shadow edges -- the culling decisions closest
// to a box -- through this kernel.
#ifndef RT_CULL_F32
#define RT_CULL_F32 1
#endif
#include <stdio.h>
#include <stdlib.h>

#include "rt_device.h"
#include "rt_ctx.h"

namespace {

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

using namespace rt;

extern "C" {

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
    rt_ctx_set_option(h.c, RT_OPT_SPECIALIZE, 0);   // one point per upload: never worth a compile
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
  RT_TRY(rt::mark_launch(c, st));
  if (!dev_out) {
    RT_HIP(hipMemcpyAsync(out, target, n * 4 * sizeof(double), hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
  }
  return RT_OK;
}

}  // extern "C"
