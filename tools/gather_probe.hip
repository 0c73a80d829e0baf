// Random-row gather ceiling of one MI355X: the HBM rate a kernel reaches when every wavefront reads whole records at
// uniformly random positions of a large array — the access pattern of an HNSW search at scale, where the rows a query
// visits are scattered over the whole index and (beyond the 256 MiB Infinity Cache) nearly every row is an HBM miss.
// The search kernels' roofline fraction is quoted against the 8 TB/s peak; this probe measures what the same pattern
// can reach at all, for the row sizes and index sizes of the BASELINE configs.
//
// Each wavefront reads `rows_per_step` rows per step, four lanes per row (the search kernels' layout: lane group g
// evaluates one neighbour, its four lanes read a quarter of the row each, 16-byte loads), for `steps` steps, with
// `depth` steps' loads in flight (depth 1: the next step's rows are requested only after this step's arrived, as a
// search's next expansion waits for its list).  Row ids are a hash of (wave, step, group), uniform over the array.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o gather_probe tools/gather_probe.hip
// Usage: gather_probe <array GiB> <row bytes> <waves per CU> <rows per step> <depth> [steps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                   \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// NC: 16-byte chunks per row (row bytes / 16, rows packed at that stride like the index's records); lane c of a group
// reads chunks c, c + 4, ... (the search kernels' interleave); DEPTH: steps in flight
template <int NC, int DEPTH>
__global__ __launch_bounds__(64) void gather(const uint4* __restrict__ a, unsigned long long n_rows, int steps,
                                             int rows_per_step, unsigned* out) {
  constexpr int CH = (NC + 3) / 4;
  const int lane = threadIdx.x, g = lane >> 2, c = lane & 3;
  const unsigned long long wave = blockIdx.x;
  const bool act = g < rows_per_step;
  uint4 buf[DEPTH][CH];
  unsigned acc = 0;
  auto issue = [&](int s, uint4* b) {
    const unsigned long long row = mix((wave << 32) ^ (static_cast<unsigned long long>(s) << 6) ^ g) % n_rows;
    const uint4* p = a + row * NC;
#pragma unroll
    for (int u = 0; u < CH; ++u) b[u] = act && 4 * u + c < NC ? p[4 * u + c] : make_uint4(0, 0, 0, 0);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) issue(d, buf[d]);
  for (int s = 0; s < steps; s += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int u = 0; u < CH; ++u) acc ^= buf[d][u].x ^ buf[d][u].y ^ buf[d][u].z ^ buf[d][u].w;
      if (s + d + DEPTH < steps) issue(s + d + DEPTH, buf[d]);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads alive
}

template <int NC>
hipError_t launch(int depth, int grid, const uint4* a, unsigned long long n_rows, int steps, int rps, unsigned* out) {
  switch (depth) {
    case 1: gather<NC, 1><<<grid, 64>>>(a, n_rows, steps, rps, out); break;
    case 2: gather<NC, 2><<<grid, 64>>>(a, n_rows, steps, rps, out); break;
    default: gather<NC, 4><<<grid, 64>>>(a, n_rows, steps, rps, out); break;
  }
  return hipGetLastError();
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s <array GiB> <row bytes> <waves per CU> <rows per step> <depth> [steps]\n", argv[0]);
    return 2;
  }
  const double gib = std::atof(argv[1]);
  const int row_bytes = std::atoi(argv[2]), wpc = std::atoi(argv[3]), rps = std::atoi(argv[4]),
            depth = std::atoi(argv[5]);
  const int steps = argc > 6 ? std::atoi(argv[6]) : 256;
  if (rps < 1 || rps > 16 || (depth != 1 && depth != 2 && depth != 4)) {
    std::fprintf(stderr, "rows per step 1-16; depth 1, 2 or 4\n");
    return 2;
  }
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const size_t bytes = static_cast<size_t>(gib * (1ull << 30)) / row_bytes * row_bytes;
  const unsigned long long n_rows = bytes / row_bytes;
  uint4* a = nullptr;
  unsigned* out = nullptr;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(a, 1, bytes));
  const int grid = prop.multiProcessorCount * wpc;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&]() -> hipError_t {
    switch (row_bytes) {
      case 192: return launch<12>(depth, grid, a, n_rows, steps, rps, out);
      case 384: return launch<24>(depth, grid, a, n_rows, steps, rps, out);
      case 400: return launch<25>(depth, grid, a, n_rows, steps, rps, out);
      case 416: return launch<26>(depth, grid, a, n_rows, steps, rps, out);
      case 448: return launch<28>(depth, grid, a, n_rows, steps, rps, out);
      case 512: return launch<32>(depth, grid, a, n_rows, steps, rps, out);
      default: return hipErrorInvalidValue;  // (the row sizes of the BASELINE configs and their paddings)
    }
  };
  CHECK(run());  // warm
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0));
    CHECK(run());
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double moved = static_cast<double>(grid) * steps * rps * row_bytes;
  std::printf("{\"array_gib\": %.2f, \"row_bytes\": %d, \"waves_per_cu\": %d, \"rows_per_step\": %d, \"depth\": %d, "
              "\"steps\": %d, \"ms\": %.4f, \"gb_per_s\": %.1f, \"frac_of_8tbs\": %.3f}\n",
              bytes / double(1ull << 30), row_bytes, wpc, rps, depth, steps, best, moved / best / 1e6,
              moved / best / 1e6 / 8000.0);
  CHECK(hipFree(a));
  CHECK(hipFree(out));
  return 0;
}
