// k_tail.hip -- the tail kernel (RT_OPT_TAIL_TILES): the costliest calibrated tiles of a tail-bound
// launch of a reflection-only scene, traced G lanes per pixel (rt_device.h tail_body: the cooperative
// nearest-hit and shadow walks, each lane testing some leaves, the group reducing), on a hardware queue
// of its own while the deferred kernel renders the rest (k_rows.hip launch_bands).
//
// A lane of the cooperative walks reads a different leaf and object record than its neighbours, so
// the scene tables cannot be scalar loads as in the other kernels; from HBM / L2 each of those
// dependent per-lane loads costs ~1-2 k cycles and the first version of this kernel took 199 us for
// 64 tiles -- longer than the launch it was to shorten (profiles/r05d_tail_kernel_trace.txt).  This
// translation unit compiles the device code with generic table pointers (RT_CAS_GENERIC) and every
// workgroup first copies the tables [objects, texels) of the blob into LDS: the walks then read them at
// LDS latency.  (For the throughput kernels, where every lane reads the same record, staging the tables
// in LDS measured 1.77x slower than scalar loads, profiles/r03q_lds_scene_ab.txt.)
#define RT_CAS_GENERIC 1
#include "rt_device.h"
#include "rt_ctx.h"

namespace {

// One wave per workgroup, 2 waves per SIMD: a few thousand waves whose latency is the point.
template <bool FC, int G>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void render_tail_kernel(
    RtDevScene S, int y_first, int band_rows, int band_pitch, int n_rows, int max_depth, uint8_t* __restrict__ out,
    size_t stride, const int32_t* __restrict__ tiles, int rgb, uint32_t tbl_bytes) {
  // The tail waves share their SIMDs with the main launch's (7 waves/SIMD of the deferred kernel), and
  // round-robin issue would stretch their latency by as much: they take the highest issue priority.
  __builtin_amdgcn_s_setprio(3);
  extern __shared__ __attribute__((aligned(16))) uint8_t s_tbl[];   // [frames | tables]
  constexpr uint32_t FRAME_BYTES = rows_lds_doubles<RT_MODE_REFL>() * 8;
  uint8_t* tbl = s_tbl + FRAME_BYTES;
  const uint8_t* src = (const uint8_t*)S.objects;                    // the blob's first table
  for (uint32_t q = threadIdx.x * 16; q < tbl_bytes; q += 64 * 16) *(uint4*)&tbl[q] = *(const uint4*)&src[q];
  __syncthreads();
  auto rebase = [&](const void* p) { return (const void*)(tbl + ((const uint8_t*)p - src)); };
  RtDevScene L = S;
  L.objects = (const RtObject*)rebase(S.objects);
  L.trav = (const RtTrav*)rebase(S.trav);
  L.strav = (const RtTrav*)rebase(S.strav);
  L.nodes = (const RtNode*)rebase(S.nodes);
  L.leaves = (const RtLeaf*)rebase(S.leaves);
  L.prog = (const RtProg*)rebase(S.prog);
  L.lights = (const RtLight*)rebase(S.lights);
  L.textures = (const RtTexture*)rebase(S.textures);
  tail_body<false, FC, G>(L, y_first, band_rows, band_pitch, n_rows, max_depth, out, stride, tiles, rgb,
                          (lds_f64*)(void*)s_tbl);
}

}  // namespace

int rt::launch_tail(rt_ctx* c, hipStream_t st, uint32_t n_tail, int a0, int a1, int a2, int a3, int max_depth,
                    uint8_t* target, size_t tstride, const int32_t* d_tail, int rgbi, bool fc) {
  const int nl = c->dev.n_leaves;
  const int G = nl <= 16 ? 16 : nl <= 32 ? 32 : 64;
  const dim3 grid(n_tail * (unsigned)G);
  const uint32_t tb = (uint32_t)c->tbl_bytes;
  const size_t lds = (size_t)rows_lds_doubles<RT_MODE_REFL>() * 8 + tb;
#define RT_LAUNCH_TAIL(FCv, Gv)                                                                                    \
  hipLaunchKernelGGL((render_tail_kernel<FCv, Gv>), grid, dim3(64), lds, st, c->dev, a0, a1, a2, a3, max_depth, target, \
                     tstride, d_tail, rgbi, tb)
  if (fc) { if (G == 16) RT_LAUNCH_TAIL(true, 16); else if (G == 32) RT_LAUNCH_TAIL(true, 32); else RT_LAUNCH_TAIL(true, 64); }
  else { if (G == 16) RT_LAUNCH_TAIL(false, 16); else if (G == 32) RT_LAUNCH_TAIL(false, 32); else RT_LAUNCH_TAIL(false, 64); }
#undef RT_LAUNCH_TAIL
  RT_HIP(hipGetLastError());
  return RT_OK;
}
