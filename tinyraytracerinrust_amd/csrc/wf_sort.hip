// wf_sort.hip -- the wavefront path's per-level ordering (render_kernels.hip "wavefront path"):
// a rocPRIM radix sort (through hipCUB) of (coherence key, slot) pairs.  Own translation unit so the
// render kernels' file does not compile the library's templates.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

// d_temp == nullptr: *temp_bytes = the scratch the sort of n pairs needs.  Sorts bits [0, end_bit).
extern "C" hipError_t rt_wf_sort_pairs(void* d_temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                       const uint32_t* vals_in, uint32_t* vals_out, int n, int end_bit,
                                       hipStream_t stream) {
  return hipcub::DeviceRadixSort::SortPairs(d_temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, end_bit,
                                            stream);
}
