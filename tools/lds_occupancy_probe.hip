// LDS allocation as the runtime's occupancy calculator sees it on gfx950: for a 64-thread kernel with no register
// pressure, the wavefronts per CU at each dynamic LDS size — the granule sizes are rounded up to, and the LDS per CU.
// The fast kernel's table sizing (capi.cc) divides the LDS per CU by its per-wave bytes; a size just past a granule
// boundary holds one wavefront fewer than that division says.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/lds_occupancy_probe tools/lds_occupancy_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k(int* o) {
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (o) o[threadIdx.x] = s[63 - threadIdx.x];
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  std::printf("{\"lds_per_cu\": %zu, \"lds_per_block\": %zu, \"cus\": %d}\n", p.maxSharedMemoryPerMultiProcessor,
              p.sharedMemPerBlock, p.multiProcessorCount);
  int last = -1;
  for (size_t b = 128; b <= 65536; b += 128) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64, b) != hipSuccess) return 2;
    if (n != last) std::printf("{\"lds_bytes\": %zu, \"waves_per_cu\": %d}\n", b, n);
    last = n;
  }
  for (size_t b : {22032ul, 23312ul, 26128ul, 27152ul, 35344ul, 39440ul, 40720ul, 41584ul}) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64, b) != hipSuccess) return 3;
    std::printf("{\"lds_bytes\": %zu, \"waves_per_cu\": %d, \"check\": true}\n", b, n);
  }
  return 0;
}
