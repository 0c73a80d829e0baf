// Device-side argument blocks and host launchers for the gfx950 kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace shine {

struct DevGraph {
  const void* vec;        // [N][dim] f32 or f16
  const uint32_t* adj0;   // [N][M0]
  const uint32_t* uid;    // [N]
  const uint32_t* up_base;// [N]
  const uint32_t* adjU;   // [R][MU]
  const uint32_t* inv_uid;// [inv_size] uid → dense id (distance-batch API)
  uint32_t inv_size;
  uint32_t N, M0, MU, ep, ep_level, lists_unique;
};

struct SearchArgs {
  DevGraph g;
  const float* queries;   // [nq_total][dim]
  const uint32_t* qmap;   // work item → query index (nullptr: identity)
  uint32_t nq;            // work items
  uint32_t k, ef, cap;    // cap: next_candidates capacity held in LDS
  uint32_t* out_ids;      // [nq_total][k]
  float* out_dists;       // [nq_total][k] (nullable)
  uint32_t* qstats;       // [nq_total][8] (nullable)
  uint32_t* visited;      // [slots][words_per_slot] bitmaps, all-zero between queries
  uint64_t words_per_slot;
  uint32_t* vlog;         // [slots][log_cap] ids whose visited bit is set (for clearing)
  uint32_t log_cap;
  uint32_t* counter;      // work queue head (zeroed before every launch)
};

struct DistArgs {
  DevGraph g;
  const float* queries;
  uint32_t nq;
  const uint32_t* node_uids;  // [nq][n_per]
  uint32_t n_per;
  float* out;                 // [nq][n_per]
};

// LDS bytes a search workgroup needs for (ef, cap).
inline size_t search_lds_bytes(uint32_t ef, uint32_t cap) { return 8ull * (ef + cap) + 64 * 4 * 2; }

bool dim_supported(uint32_t dim, int elem);

// Returns hipSuccess or the launch error.  grid = number of persistent search slots (one wavefront each).
hipError_t launch_search(uint32_t dim, int metric, int elem, uint32_t grid, const SearchArgs& a, hipStream_t s);
hipError_t launch_distance(uint32_t dim, int metric, int elem, const DistArgs& a, hipStream_t s);

}  // namespace shine
