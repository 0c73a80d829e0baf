// Host distances in the FP order of the GPU kernels and the oracle (DESIGN.md "Distance FP order"): 8 lane
// accumulators over the 16-aligned prefix (lane j: elements i ≡ j mod 8, FMA chain), a left-to-right sum of the
// lanes, then the scalar tail (distance.hh:11-151).  Used by the builder and the region planner.
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
#define SHINE_HOST_AVX2 1
#endif

namespace shine {

inline float host_l2(const float* a, const float* b, uint32_t dim) {
  const uint32_t q16 = dim >> 4 << 4;
  alignas(32) float acc[8];
#ifdef SHINE_HOST_AVX2
  __m256 s = _mm256_setzero_ps();
  for (uint32_t i = 0; i < q16; i += 8) {
    const __m256 d = _mm256_sub_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i));
    s = _mm256_fmadd_ps(d, d, s);
  }
  _mm256_store_ps(acc, s);
#else
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (uint32_t i = 0; i < q16; i += 8)
    for (int j = 0; j < 8; ++j) {
      const float d = a[i + j] - b[i + j];
      acc[j] = std::fmaf(d, d, acc[j]);
    }
#endif
  float r = acc[0];
  for (int j = 1; j < 8; ++j) r = r + acc[j];
  for (uint32_t i = q16; i < dim; ++i) {
    const float d = a[i] - b[i];
    r = std::fmaf(d, d, r);
  }
  return r;
}

inline float host_ip(const float* a, const float* b, uint32_t dim) {
  const uint32_t q16 = dim >> 4 << 4;
  alignas(32) float acc[8];
#ifdef SHINE_HOST_AVX2
  __m256 s = _mm256_setzero_ps();
  for (uint32_t i = 0; i < q16; i += 8) s = _mm256_fmadd_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i), s);
  _mm256_store_ps(acc, s);
#else
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (uint32_t i = 0; i < q16; i += 8)
    for (int j = 0; j < 8; ++j) acc[j] = std::fmaf(a[i + j], b[i + j], acc[j]);
#endif
  float r = acc[0];
  for (int j = 1; j < 8; ++j) r = r + acc[j];
  float t = 0.f;
  for (uint32_t i = q16; i < dim; ++i) t = std::fmaf(a[i], b[i], t);
  return 1.0f - (r + t);
}

// metric 0 = L2 (L2Distance), 1 = inner product (IPDistance: 1 - <a, b>)
inline float host_dist(int metric, const float* a, const float* b, uint32_t dim) {
  return metric == 0 ? host_l2(a, b, dim) : host_ip(a, b, dim);
}

}  // namespace shine
