// Dispatch over the compiled vector dimensions (one kernels_dim.hip translation unit per dimension) and the
// diagnostics kernel.  Device code: kernels_impl.h.
#include "kernels_impl.h"

namespace shine {


bool dim_supported(uint32_t dim, int elem) {
#define SHINE_CASE(DD) \
  if (dim == DD) return true;
  if (elem == 0) {
    SHINE_DIMS(SHINE_CASE)
  } else if (elem == 1) {
    return dim == 96 || dim == 128 || dim == 200;
  } else if (elem_is_byte(elem)) {
    SHINE_BYTE_DIMS(SHINE_CASE)
  }
#undef SHINE_CASE
  return false;
}

hipError_t launch_search(uint32_t dim, int metric, int elem, uint32_t grid, const SearchArgs& a, hipStream_t s) {
  if (elem_is_byte(elem)) {
#define SHINE_CASE(DD)                                                                                     \
  if (dim == DD)                                                                                           \
    return elem == 2 ? launch_search_d##DD##_e2(metric, grid, a, s) : launch_search_d##DD##_e3(metric, grid, a, s);
    SHINE_BYTE_DIMS(SHINE_CASE)
#undef SHINE_CASE
    return hipErrorInvalidValue;
  }
#define SHINE_CASE(DD) \
  if (dim == DD) return launch_search_d##DD(metric, elem, grid, a, s);
  SHINE_DIMS(SHINE_CASE)
#undef SHINE_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_distance(uint32_t dim, int metric, int elem, const DistArgs& a, hipStream_t s) {
  if (elem_is_byte(elem)) {
#define SHINE_CASE(DD) \
  if (dim == DD) return elem == 2 ? launch_distance_d##DD##_e2(metric, a, s) : launch_distance_d##DD##_e3(metric, a, s);
    SHINE_BYTE_DIMS(SHINE_CASE)
#undef SHINE_CASE
    return hipErrorInvalidValue;
  }
#define SHINE_CASE(DD) \
  if (dim == DD) return launch_distance_d##DD(metric, elem, a, s);
  SHINE_DIMS(SHINE_CASE)
#undef SHINE_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_heap_replay(int is_max, const int32_t* ops, const float* vals, const uint32_t* ids, uint32_t n_ops,
                              uint32_t k, float* out_d, uint32_t* out_ids, uint32_t* out_n, hipStream_t s) {
  const size_t lds = 8ull * (n_ops + 1);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const void* kern = is_max ? reinterpret_cast<const void*>(&heap_replay_kernel<true>)
                            : reinterpret_cast<const void*>(&heap_replay_kernel<false>);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return e;
  }
  if (is_max)
    hipLaunchKernelGGL(heap_replay_kernel<true>, dim3(1), dim3(64), lds, s, ops, vals, ids, n_ops, k, out_d, out_ids,
                       out_n);
  else
    hipLaunchKernelGGL(heap_replay_kernel<false>, dim3(1), dim3(64), lds, s, ops, vals, ids, n_ops, k, out_d, out_ids,
                       out_n);
  return hipGetLastError();
}

}  // namespace shine
