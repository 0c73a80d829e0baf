// Dimension-independent kernels of the GPU batch builder (gpu_build.cc): row layout conversion, id tables, the
// request sort (rocPRIM radix sort) and its segment starts.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "kernels.h"

namespace shine {
namespace {

__global__ __launch_bounds__(256) void iota_kernel(uint32_t* out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += static_cast<uint64_t>(gridDim.x) * 256ull)
    out[i] = static_cast<uint32_t>(i);
}

// one thread per (row, component); grid-stride
__global__ __launch_bounds__(256) void rows_kernel(const float* __restrict__ src, void* __restrict__ dst, uint64_t n,
                                                   uint32_t dim, int elem, int from_dev, uint64_t rowb) {
  const uint64_t total = n * dim;
  for (uint64_t x = blockIdx.x * 256ull + threadIdx.x; x < total; x += static_cast<uint64_t>(gridDim.x) * 256ull) {
    const uint64_t r = x / dim;
    const uint32_t i = static_cast<uint32_t>(x - r * dim);
    const float v = src[r * dim + (from_dev ? permuted_index(dim, i) : i)];
    if (elem == 0) {
      static_cast<float*>(dst)[r * dim + permuted_index(dim, i)] = v;
    } else if (elem == 1) {
      static_cast<__half*>(dst)[r * dim + i] = __float2half(v);  // fp16 rows: natural order (kernels.h)
    } else {
      static_cast<uint8_t*>(dst)[r * rowb + permuted_index_bytes(dim, i)] =
          static_cast<uint8_t>(static_cast<int>(v));
    }
  }
}

__global__ __launch_bounds__(256) void segments_kernel(const uint32_t* __restrict__ key, uint32_t n, uint32_t none,
                                                       uint32_t* __restrict__ seg, uint32_t* nseg) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = key[i];
  if (k < none && (i == 0 || key[i - 1] != k)) seg[atomicAdd(nseg, 1u)] = i;
}

// a batch's level-0 searches: distcomps summed into out[0], searches that ended with a status counted in out[1]
__global__ __launch_bounds__(256) void qstats_kernel(const uint32_t* __restrict__ qs, uint32_t nq,
                                                     unsigned long long* out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  unsigned long long d = 0, f = 0;
  if (i < nq) {
    d = qs[static_cast<uint64_t>(i) * kQsWords];
    f = qs[static_cast<uint64_t>(i) * kQsWords + 6] != 0u ? 1ull : 0ull;
  }
  for (int o = 32; o > 0; o >>= 1) {
    d += __shfl_xor(d, o);
    f += __shfl_xor(f, o);
  }
  if ((threadIdx.x & 63) == 0 && (d || f)) {
    atomicAdd(&out[0], d);
    atomicAdd(&out[1], f);
  }
}

// out[0] = 1 if a component (f32, device layout) is not exactly a byte value of the kind (u8: elem 2, i8: elem 3)
__global__ __launch_bounds__(256) void fits_bytes_kernel(const float* __restrict__ src, uint64_t total, int elem,
                                                         uint32_t* out) {
  const float lo = elem == 2 ? 0.f : -128.f, hi = elem == 2 ? 255.f : 127.f;
  bool bad = false;
  for (uint64_t x = blockIdx.x * 256ull + threadIdx.x; x < total; x += static_cast<uint64_t>(gridDim.x) * 256ull) {
    const float v = src[x];
    const float r = static_cast<float>(static_cast<int>(v));
    bad |= !(v >= lo && v <= hi) || __float_as_uint(v) != __float_as_uint(r);
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(out, 1u);
}

uint32_t grid_for(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return static_cast<uint32_t>(g < 65536 ? (g ? g : 1) : 65536);
}

}  // namespace

hipError_t launch_iota(uint32_t* out, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n)), dim3(256), 0, s, out, n);
  return hipGetLastError();
}

hipError_t launch_rows_to_device(const float* src, void* dst, uint64_t n, uint32_t dim, int elem, bool from_device_layout,
                                 hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (elem < 0 || elem > 3) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_kernel, dim3(grid_for(n * dim)), dim3(256), 0, s, src, dst, n, dim, elem,
                     from_device_layout ? 1 : 0, row_bytes(dim, elem));
  return hipGetLastError();
}

hipError_t launch_qstats_sum(const uint32_t* qs, uint32_t nq, unsigned long long* out, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  hipLaunchKernelGGL(qstats_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, qs, nq, out);
  return hipGetLastError();
}

hipError_t launch_fits_bytes(const float* src, uint64_t total, int elem, uint32_t* flag, hipStream_t s) {
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(fits_bytes_kernel, dim3(grid_for(total)), dim3(256), 0, s, src, total, elem, flag);
  return hipGetLastError();
}

hipError_t launch_segments(const uint32_t* skey, uint32_t n, uint32_t key_none, uint32_t* seg, uint32_t* nseg,
                           hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(segments_kernel, dim3((n + 255) / 256), dim3(256), 0, s, skey, n, key_none, seg, nseg);
  return hipGetLastError();
}

hipError_t radix_sort_u32_pairs(void* temp, size_t* temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                const uint32_t* vals_in, uint32_t* vals_out, uint32_t n, uint32_t bits, hipStream_t s) {
  size_t bytes = temp ? *temp_bytes : 0;
  const hipError_t e = rocprim::radix_sort_pairs(temp, bytes, keys_in, keys_out, vals_in, vals_out, n, 0u, bits, s);
  if (!temp) *temp_bytes = bytes;
  return e;
}

}  // namespace shine
