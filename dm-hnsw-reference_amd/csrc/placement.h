// Region placement (balanced k-means over the top levels) and adaptive balanced query routing; see placement.cc.
#pragma once

#include <cstdint>
#include <functional>
#include <vector>

#include "graph.h"

namespace shine {

constexpr uint32_t kKmeansIterationLimit = 1000;  // kmeans.hh:12
constexpr uint32_t kFetchLevelNodes = 500;        // placement.hh:29
constexpr uint32_t kLimitPerCn = 200;             // constants.hh:25

// The points k-means runs over: rows of dim floats, in the order fetch_level yields them.
struct KmeansInput {
  int metric = 0;  // 0 = L2Distance, 1 = IPDistance
  uint32_t dim = 0;
  std::vector<const float*> rows;
};

struct KmeansResult {
  std::vector<float> centroids;      // [k][dim]
  std::vector<uint32_t> assignment;  // cluster of every row
  std::vector<uint64_t> sizes;       // rows per cluster
  uint32_t iterations = 0;
  float error = 0.f;
};

// Kmeans::run_kmeans (kmeans.hh:93-137).  Needs rows.size() >= k.
KmeansResult run_kmeans(const KmeansInput& in, uint32_t k);
// Kmeans::balanced_kmeans (kmeans.hh:259-377): moves rows between the clusters of r in place and returns the
// sizes of the final nearest-centroid partition (the "actual" sizes).
std::vector<uint64_t> balanced_kmeans(const KmeansInput& in, uint32_t k, float c, float penalty_factor,
                                      uint32_t max_cluster_size_difference, KmeansResult& r, uint32_t* iterations);

struct Regions {
  uint32_t k = 0, dim = 0;        // k regions: one per GPU slot (the reference: one per compute node)
  int metric = 0;
  std::vector<float> centroids;   // [n_centroids()][dim]: 2k centroids when k is odd (run_and_optimize)
  std::vector<uint32_t> mapping;  // centroid -> region
  std::vector<uint64_t> sizes;    // rows of the k-means input per region after balancing
  uint32_t iterations = 0, balance_iterations = 0;
  uint32_t n_centroids() const { return static_cast<uint32_t>(mapping.size()); }
};

// Kmeans::run_and_optimize (kmeans.hh:24-91): balanced k-means with k (even) or 2k clusters whose closest pairs
// are merged (odd k).  balanced = false is the plain run_kmeans branch of Placement (placement.hh:45-58).
// Returns 0, or -1 when there are fewer rows than clusters (the reference asserts).
int run_and_optimize(const KmeansInput& in, uint32_t k, bool balanced, Regions& out);

// Placement::fetch_level (placement.hh:78-106): breadth-first over the lists of the top level from the entry
// point, one level lower until at least min_nodes were found.
std::vector<uint32_t> top_level_sample(const HostGraph& G, uint32_t min_nodes);
// fetch_level(500) + run_and_optimize over the sampled records' vectors.
int plan_regions(const HostGraph& G, uint32_t k, bool balanced, Regions& out);

// Placement::closest_centroids (placement.hh:63-72): the regions in the pop order of its MinPlacement heap.
void closest_regions(const Regions& R, const float* x, std::vector<uint32_t>& order);
uint32_t nearest_region(const Regions& R, const float* x);

// Owner region of every dense id (the GPU node's addition: records live in the HBM of their region's GPU).  Each
// record takes the first region of its closest_regions order below ceil(N/k * (1 + slack)) records.
std::vector<uint32_t> assign_regions(const HostGraph& G, const Regions& R, double slack, uint32_t seed);

// QueryRouter's routing state (query_router.hh:37-50, 413-416) and its run_routing loop (280-387) without the
// transport: queries go to their closest region whose per-batch histogram is below its limit (BALANCED_ROUTING);
// every batch_size = kLimitPerCn * k queries the histogram is cleared and, with adaptive routing, the limits are
// re-derived from the compute nodes' queue sizes (update_limits, 106-151).  The state lives across calls, as the
// reference's router lives for the whole query phase.
struct Router {
  uint32_t k = 0;
  uint64_t batch_size = 0;
  uint64_t local_slot = 0;  // queries routed so far
  bool adaptive = true;     // ADAPTIVE_ROUTING (constants.hh:21)
  std::vector<uint64_t> limits, histogram;

  void init(uint32_t regions);
  // update_limits: false (limits kept) when the progresses sum to less than k
  bool update_limits(const std::vector<uint32_t>& progresses);
  // Route nq queries (rows of stride floats).  progress(routed, queue_sizes) is asked for the k queue sizes at
  // every batch boundary; routed[r] = queries of this call routed to region r so far.
  void route(const Regions& R, const float* q, uint32_t nq, uint64_t stride,
             const std::function<void(const std::vector<uint64_t>& routed, std::vector<uint32_t>& progress)>& progress,
             uint32_t* out);
};

}  // namespace shine
