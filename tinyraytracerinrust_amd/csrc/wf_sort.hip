// wf_sort.hip -- the wavefront path's orderings (k_wavefront.hip): the in-tree bucket sort below
// orders the pair path's (object, pair) lists, its hit points, and the non-pair levels' rays by the
// top 12 bits of their coherence key.  (Diagnostic builds with RT_WF_RADIX_SORT keep the rocPRIM radix
// sort through hipCUB the non-pair levels used before round 4, for A/B runs.)
#include <hip/hip_runtime.h>
#ifdef RT_WF_RADIX_SORT
#include <hipcub/hipcub.hpp>
#endif
#include <stdint.h>
#include <algorithm>

#ifdef RT_WF_RADIX_SORT
// d_temp == nullptr: *temp_bytes = the scratch the sort of n pairs needs.  Sorts bits [0, end_bit).
extern "C" hipError_t rt_wf_sort_pairs(void* d_temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                       const uint32_t* vals_in, uint32_t* vals_out, int n, int end_bit,
                                       hipStream_t stream) {
  return hipcub::DeviceRadixSort::SortPairs(d_temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit,
                                            stream);
}
#endif

// ---------------------------------------------------------------------------- bucket sort
// The pair path's sort of (object, pair) by object: few keys (the scene's objects), many items.  A
// counting sort in three launches at most (a radix sort of a few million items takes a dozen: rocPRIM's
// block sort + merge passes below its one-sweep size), not stable -- the pair order within an
// object does not matter (k_wavefront.hip wfp_*: the folds are atomic min / add / or).
//   hist:    per workgroup an LDS histogram of its grid-stride share, added to cnt[] (one atomic per
//            nonzero bin and workgroup);
//   scan:    one workgroup turns cnt[] into exclusive offsets in place (a launch of its own: fusing it
//            into hist's last workgroup needs a device-scope fence per workgroup, which writes back
//            the L2s of the 8 XCDs -- measured 3.6x slower hist, profiles/r05z_wavefront_round4.txt);
//   scatter: per workgroup a contiguous chunk: LDS counts give each item its rank among the chunk's
//            items of its key, one atomic per nonzero bin reserves the chunk's run in that bucket.
// Sorts of at most RT_BS_FUSED_BINS bins (the pair lists: one bin per object; the hit points) skip the
// scan launch: every scatter workgroup scans the counts itself in LDS (2 K words at most) and reserves
// its runs on a second, zeroed word per bin (cnt[RT_BS_FUSED_BINS + b]): a launch boundary costs
// 4-6 us on the pair path's small levels (profiles/r07k_fractal_kernel_stats.csv), the scan of 2 K
// words a fraction of one.
#define RT_BS_MAX_BINS 4096
#define RT_BS_FUSED_BINS 2048
#define RT_BS_THREADS 256
#define RT_BS_PER_THREAD 16
__device__ __forceinline__ uint32_t rt_bs_bin(uint32_t key, int shift, uint32_t nb) {
  return min(key >> shift, nb - 1u);
}
// n_dev != nullptr: the item count is min(*n_dev, n) (a count another kernel wrote: no host read)
__global__ __launch_bounds__(RT_BS_THREADS) void rt_bs_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                           const uint32_t* __restrict__ n_dev, uint32_t nb, int shift,
                                                           uint32_t* __restrict__ cnt) {
  if (n_dev) n = min(*n_dev, n);
  // contiguous chunks of RT_BS_THREADS x RT_BS_PER_THREAD items, as the scatter takes them: a workgroup
  // past the count leaves at once, and every thread issues its chunk's loads before its LDS atomics.
  // (Round 5's first form strode the whole grid over the items: on the pair path's device-driven levels
  // the grid is sized for the lists' capacity, and 1024 workgroups each added ~all bins to cnt[] --
  // 13-20 us of same-address atomics for a 100-640 k item level, profiles/r07r_fractal_levels_trace.txt.)
  constexpr uint32_t CH = RT_BS_THREADS * RT_BS_PER_THREAD;
  if (blockIdx.x * CH >= n) return;
  __shared__ uint32_t h[RT_BS_MAX_BINS];
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  for (uint32_t base = blockIdx.x * CH; base < n; base += gridDim.x * CH) {
    uint32_t k[RT_BS_PER_THREAD];
#pragma unroll
    for (int e = 0; e < RT_BS_PER_THREAD; ++e) {
      const uint32_t i = base + (uint32_t)e * RT_BS_THREADS + threadIdx.x;
      k[e] = i < n ? keys[i] : 0xffffffffu;
    }
#pragma unroll
    for (int e = 0; e < RT_BS_PER_THREAD; ++e)
      if (base + (uint32_t)e * RT_BS_THREADS + threadIdx.x < n) atomicAdd(&h[rt_bs_bin(k[e], shift, nb)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&cnt[b], h[b]);
}

__global__ __launch_bounds__(1024) void rt_bs_scan(uint32_t* __restrict__ cnt, uint32_t nb) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) s += cnt[b];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {          // inclusive scan of the thread sums
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) {
    const uint32_t c = cnt[b];
    cnt[b] = run;
    run += c;
  }
}

__global__ __launch_bounds__(RT_BS_THREADS) void rt_bs_scatter(const uint32_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ vals, uint32_t n,
                                                              const uint32_t* __restrict__ n_dev, uint32_t nb,
                                                              int shift, uint32_t* __restrict__ off,
                                                              uint32_t* __restrict__ keys_out,
                                                              uint32_t* __restrict__ vals_out, int fused) {
  const uint32_t cap = n;                                    // the output lists' capacity
  if (n_dev) n = min(*n_dev, n);
  __shared__ uint32_t h[RT_BS_MAX_BINS];
  __shared__ uint32_t pre[RT_BS_FUSED_BINS];                 // fused: the exclusive offsets of the bins
  constexpr uint32_t CH = RT_BS_THREADS * RT_BS_PER_THREAD;
  if (blockIdx.x * CH >= n) return;
  // a chunk's keys and values are loaded before the work that does not need them (the first chunk's
  // during the fused scan, the next chunk's after this one's stores are issued): the small levels'
  // scatters are latency chains
  uint32_t k[RT_BS_PER_THREAD], v[RT_BS_PER_THREAD], r[RT_BS_PER_THREAD];
  auto load = [&](uint32_t base) {
#pragma unroll
    for (int e = 0; e < RT_BS_PER_THREAD; ++e) {
      const uint32_t i = base + (uint32_t)e * RT_BS_THREADS + threadIdx.x;
      k[e] = i < n ? rt_bs_bin(keys[i], shift, nb) : 0u;
      v[e] = i < n ? vals[i] : 0u;
    }
  };
  uint32_t base = blockIdx.x * CH;
  load(base);
  if (fused) {                                               // off[] holds the counts: scan them here
    constexpr uint32_t PER = RT_BS_FUSED_BINS / RT_BS_THREADS;
    const uint32_t b0 = threadIdx.x * PER;
    uint32_t c[PER], s = 0;
#pragma unroll
    for (uint32_t e = 0; e < PER; ++e) {
      c[e] = b0 + e < nb ? off[b0 + e] : 0u;
      s += c[e];
    }
    h[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t o = 1; o < RT_BS_THREADS; o <<= 1) {        // inclusive scan of the thread sums
      const uint32_t a = threadIdx.x >= o ? h[threadIdx.x - o] : 0u;
      __syncthreads();
      h[threadIdx.x] += a;
      __syncthreads();
    }
    uint32_t run = h[threadIdx.x] - s;
#pragma unroll
    for (uint32_t e = 0; e < PER; ++e) {
      pre[b0 + e] = run;
      run += c[e];
    }
    __syncthreads();
  }
  uint32_t* const cur = off + RT_BS_FUSED_BINS;
  while (true) {                                             // chunks, grid-stride
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < RT_BS_PER_THREAD; ++e) {
      const uint32_t i = base + (uint32_t)e * RT_BS_THREADS + threadIdx.x;
      r[e] = i < n ? atomicAdd(&h[k[e]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
      if (h[b]) h[b] = fused ? pre[b] + atomicAdd(&cur[b], h[b]) : atomicAdd(&off[b], h[b]);   // this chunk's run in bucket b
    __syncthreads();
#pragma unroll
    for (int e = 0; e < RT_BS_PER_THREAD; ++e) {
      const uint32_t i = base + (uint32_t)e * RT_BS_THREADS + threadIdx.x;
      if (i < n) {
        // (q < cap: the counts are those of the stored items; the bound guards the lists regardless)
        const uint32_t q = h[k[e]] + r[e];
        if (q < cap) {
          keys_out[q] = k[e];
          vals_out[q] = v[e];
        }
      }
    }
    base += gridDim.x * CH;
    if (base >= n) break;
    __syncthreads();
    load(base);
  }
}

// Sorts n (key, value) pairs by bin = min(key >> shift, nb - 1) (nb <= RT_BS_MAX_BINS) into keys_out
// (the bins) / vals_out; cnt: device scratch of nb words, or 2 x RT_BS_FUSED_BINS words when nb <=
// RT_BS_FUSED_BINS (the fused scan's counts and run cursors).  n_dev != nullptr: the count is
// min(*n_dev, n), read on the device (n is then the capacity the grids are sized for).  zero_cnt =
// false: the caller already zeroed that scratch on this stream.  counted: the kernel that wrote the
// keys also added their bins' counts into cnt[0, nb) (no histogram launch; the fused scan only).
extern "C" hipError_t rt_wf_bucket_sort(const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                                        uint32_t* vals_out, uint32_t n, const uint32_t* n_dev, uint32_t nb, int shift,
                                        uint32_t* cnt, bool zero_cnt, hipStream_t stream, bool counted) {
  if (nb == 0 || nb > RT_BS_MAX_BINS) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const int fused = nb <= RT_BS_FUSED_BINS ? 1 : 0;
  if (counted && (!fused || zero_cnt)) return hipErrorInvalidValue;
  if (zero_cnt) {
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)(fused ? 2 * RT_BS_FUSED_BINS : nb) * 4, stream);
    if (e != hipSuccess) return e;
  }
  const uint32_t chunk = RT_BS_THREADS * RT_BS_PER_THREAD, gc = (n + chunk - 1) / chunk;
  if (!counted)
    hipLaunchKernelGGL(rt_bs_hist, dim3(std::min<uint32_t>(gc, 1024u)), dim3(RT_BS_THREADS), 0, stream, keys_in, n, n_dev,
                       nb, shift, cnt);
  if (!fused) hipLaunchKernelGGL(rt_bs_scan, dim3(1), dim3(1024), 0, stream, cnt, nb);
  hipLaunchKernelGGL(rt_bs_scatter, dim3(std::min<uint32_t>(gc, 2048u)), dim3(RT_BS_THREADS), 0, stream, keys_in,
                     vals_in, n, n_dev, nb, shift, cnt, keys_out, vals_out, fused);
  return hipGetLastError();
}
