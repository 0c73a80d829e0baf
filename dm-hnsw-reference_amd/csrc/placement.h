// Region placement (k-means over the top levels) and balanced query routing; see placement.cc.
#pragma once

#include <cstdint>
#include <vector>

#include "graph.h"

namespace shine {

struct Regions {
  uint32_t k = 0, dim = 0;
  int metric = 0;
  std::vector<float> centroids;  // [k][dim]
};

float region_dist(int metric, const float* a, const float* b, uint32_t dim);
std::vector<uint32_t> top_level_sample(const HostGraph& G, uint32_t min_nodes);
Regions kmeans_regions(const HostGraph& G, const std::vector<uint32_t>& sample, uint32_t k, uint32_t seed);
uint32_t nearest_region(const Regions& R, const float* x);
// owner region of every dense id; each region holds at most ceil(N/k * (1 + slack)) records
std::vector<uint32_t> assign_regions(const HostGraph& G, const Regions& R, double slack, uint32_t seed);
// region of every query of a batch; each region takes at most ceil(nq/k * (1 + slack)) of them
void route_queries(const Regions& R, const float* q, uint32_t nq, double slack, uint32_t* out);

}  // namespace shine
