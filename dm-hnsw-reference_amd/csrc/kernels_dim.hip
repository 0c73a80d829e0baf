// One vector dimension's kernel instantiations (built once per dimension with -DSHINE_DIM=D; see kernels.h), or,
// with -DSHINE_BYTES=2 / 3, that dimension's byte-row (u8 / i8) instantiations.
#include "kernels_impl.h"
#ifndef SHINE_BYTES
#include "build_impl.h"
#endif

#ifndef SHINE_DIM
#error "build with -DSHINE_DIM=<dimension>"
#endif

#define SHINE_CAT2(a, b) a##b
#define SHINE_CAT(a, b) SHINE_CAT2(a, b)
#define SHINE_CAT4(a, b, c, d) SHINE_CAT(SHINE_CAT(a, b), SHINE_CAT(c, d))

namespace shine {

#ifdef SHINE_BYTES
#if SHINE_BYTES == 2
using ByteE = uint8_t;
#else
using ByteE = int8_t;
#endif

hipError_t SHINE_CAT4(launch_search_d, SHINE_DIM, _e, SHINE_BYTES)(int metric, uint32_t grid, const SearchArgs& a,
                                                                  hipStream_t s) {
  return metric == 0 ? launch_search_t<SHINE_DIM, 0, ByteE>(grid, a, s) : launch_search_t<SHINE_DIM, 1, ByteE>(grid, a, s);
}

hipError_t SHINE_CAT4(launch_distance_d, SHINE_DIM, _e, SHINE_BYTES)(int metric, const DistArgs& a, hipStream_t s) {
  return metric == 0 ? launch_distance_t<SHINE_DIM, 0, ByteE>(a, s) : launch_distance_t<SHINE_DIM, 1, ByteE>(a, s);
}

#else

hipError_t SHINE_CAT(launch_search_d, SHINE_DIM)(int metric, int elem, uint32_t grid, const SearchArgs& a,
                                                 hipStream_t s) {
  if (elem == 0)
    return metric == 0 ? launch_search_t<SHINE_DIM, 0, float>(grid, a, s) : launch_search_t<SHINE_DIM, 1, float>(grid, a, s);
#if SHINE_DIM == 96 || SHINE_DIM == 128 || SHINE_DIM == 200
  if (elem == 1)
    return metric == 0 ? launch_search_t<SHINE_DIM, 0, __half>(grid, a, s)
                       : launch_search_t<SHINE_DIM, 1, __half>(grid, a, s);
#endif
  return hipErrorInvalidValue;
}

hipError_t SHINE_CAT(launch_distance_d, SHINE_DIM)(int metric, int elem, const DistArgs& a, hipStream_t s) {
  if (elem == 0)
    return metric == 0 ? launch_distance_t<SHINE_DIM, 0, float>(a, s) : launch_distance_t<SHINE_DIM, 1, float>(a, s);
#if SHINE_DIM == 96 || SHINE_DIM == 128 || SHINE_DIM == 200
  if (elem == 1)
    return metric == 0 ? launch_distance_t<SHINE_DIM, 0, __half>(a, s) : launch_distance_t<SHINE_DIM, 1, __half>(a, s);
#endif
  return hipErrorInvalidValue;
}

hipError_t SHINE_CAT(launch_build_d, SHINE_DIM)(int which, int metric, uint32_t grid, const BuildArgs& a,
                                                hipStream_t s) {
  return metric == 0 ? launch_build_t<SHINE_DIM, 0>(which, grid, a, s) : launch_build_t<SHINE_DIM, 1>(which, grid, a, s);
}

#endif

}  // namespace shine
