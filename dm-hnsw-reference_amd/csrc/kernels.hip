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

hipError_t launch_build(uint32_t dim, int metric, int which, uint32_t grid, const BuildArgs& a, hipStream_t s) {
#define SHINE_CASE(DD) \
  if (dim == DD) return launch_build_d##DD(which, metric, grid, a, s);
  SHINE_DIMS(SHINE_CASE)
#undef SHINE_CASE
  return hipErrorInvalidValue;
}

namespace {

__global__ __launch_bounds__(256) void cache_drop_kernel(const uint32_t* ids, uint32_t n, uint32_t* cslot,
                                                         uint32_t* cbits) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) {
    const uint32_t x = ids[i];
    cslot[x] = 0xFFFFFFFFu;
    atomicAnd(&cbits[x >> 5], ~(1u << (x & 31)));
  }
}

// one workgroup per admitted record: its row into the arena slot (4-byte words; rows are whole words), then cslot (the
// slot, not cooling) and the slot's occupant
__global__ __launch_bounds__(64) void cache_fill_kernel(const uint32_t* pairs, uint32_t* cslot, uint32_t* cbits,
                                                        uint8_t* cvec, uint32_t* rlogged, uint32_t* slot_id,
                                                        const uint8_t* vec, uint64_t row_bytes) {
  const uint32_t slot = pairs[2 * blockIdx.x], id = pairs[2 * blockIdx.x + 1];
  const uint32_t* src = reinterpret_cast<const uint32_t*>(vec + static_cast<uint64_t>(id) * row_bytes);
  uint32_t* dst = reinterpret_cast<uint32_t*>(cvec + static_cast<uint64_t>(slot) * row_bytes);
  for (uint64_t w = threadIdx.x; w < row_bytes / 4; w += 64) dst[w] = src[w];
  if (threadIdx.x == 0) {
    cslot[id] = slot;
    atomicOr(&cbits[id >> 5], 1u << (id & 31));
    rlogged[slot] = 0xFFFFFFFFu;  // a new occupant: its first cooling hit of the epoch is logged
    slot_id[slot] = id;
  }
}

// the cooling flags: the arena's flag array, and bit 31 of the occupant's cslot word (the search kernels read the flag
// with the slot, kernels_impl.h kCool)
__global__ __launch_bounds__(256) void cache_cool_kernel(const uint32_t* pairs, uint32_t n, uint32_t* cool,
                                                         const uint32_t* slot_id, uint32_t* cslot) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) {
    const uint32_t slot = pairs[2 * i], flag = pairs[2 * i + 1];
    cool[slot] = flag;
    const uint32_t id = slot_id[slot];
    if (id != 0xFFFFFFFFu && (cslot[id] & 0x7FFFFFFFu) == slot) cslot[id] = slot | (flag ? 0x80000000u : 0u);
  }
}

}  // namespace

hipError_t launch_cache_apply(const uint32_t* upd, uint32_t n_drop, uint32_t n_fill, uint32_t n_cool, uint32_t* cslot,
                              uint32_t* cbits, uint8_t* cvec, uint32_t* cool, uint32_t* rlogged, uint32_t* slot_id,
                              const uint8_t* vec, uint64_t row_bytes, hipStream_t s) {
  // drops before fills (a record may leave one slot and enter another in the same update: its bit ends set)
  if (n_drop)
    hipLaunchKernelGGL(cache_drop_kernel, dim3((n_drop + 255) / 256), dim3(256), 0, s, upd, n_drop, cslot, cbits);
  if (n_fill)
    hipLaunchKernelGGL(cache_fill_kernel, dim3(n_fill), dim3(64), 0, s, upd + n_drop, cslot, cbits, cvec, rlogged, slot_id,
                       vec, row_bytes);
  if (n_cool)
    hipLaunchKernelGGL(cache_cool_kernel, dim3((n_cool + 255) / 256), dim3(256), 0, s, upd + n_drop + 2 * n_fill,
                       n_cool, cool, slot_id, cslot);
  return hipGetLastError();
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
