// Region placement of a sharded index and query routing: the GPU-node form of the reference's Placement / Kmeans /
// QueryRouter (src/cache/placement.hh:22-72, src/cache/kmeans.hh:24-377, src/router/query_router.hh:280-387).
//
// The reference clusters the top-level nodes with k-means and routes every query to the compute node whose centroid
// is closest, within per-batch limits, so that each node's cache serves one region of the space.  Here the k
// regions are the GPU slots of a sharded index: every record is owned by the slot of its region, and a query routed
// to its region reads mostly that GPU's own HBM.  Host code, run once at open and per batch for routing.
#include "placement.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>
#include <thread>

namespace shine {

float region_dist(int metric, const float* a, const float* b, uint32_t dim) {
  float s = 0.f;
  if (metric == 0) {
    for (uint32_t i = 0; i < dim; ++i) {
      const float t = a[i] - b[i];
      s += t * t;
    }
    return s;
  }
  for (uint32_t i = 0; i < dim; ++i) s += a[i] * b[i];
  return 1.f - s;
}

// Breadth-first over the lists of the top level from the entry point, one level lower while fewer than min_nodes
// were found (placement.hh:78-106 fetches the same set over RDMA).  Level 0 is used when the upper levels are small.
std::vector<uint32_t> top_level_sample(const HostGraph& G, uint32_t min_nodes) {
  std::vector<uint32_t> nodes{G.ep};
  std::vector<uint8_t> seen(G.N, 0);
  seen[G.ep] = 1;
  const uint32_t M = G.L.M, M0 = 2 * G.L.M;
  for (int level = static_cast<int>(G.ep_level); level >= 0; --level) {
    for (size_t it = 0; it < nodes.size(); ++it) {
      const uint32_t n = nodes[it];
      if (G.level[n] < static_cast<uint32_t>(level)) continue;
      const uint32_t* lst = level == 0 ? &G.adj0[static_cast<uint64_t>(n) * M0]
                                       : &G.adjU[(static_cast<uint64_t>(G.up_base[n]) + level - 1) * M];
      const uint32_t cap = level == 0 ? M0 : M;
      for (uint32_t j = 0; j < cap; ++j) {
        const uint32_t x = lst[j];
        if (x == kInvalid || seen[x]) continue;
        seen[x] = 1;
        nodes.push_back(x);
      }
    }
    if (nodes.size() >= min_nodes) break;
  }
  return nodes;
}

// Lloyd's iterations from a k-means++ seeding (fixed seed), until the centroids move less than 1e-3 in total
// (kmeans.hh:93-137 uses the same stopping rule).  Centroids are plain means (for IP too).
Regions kmeans_regions(const HostGraph& G, const std::vector<uint32_t>& sample, uint32_t k, uint32_t seed) {
  Regions R;
  R.k = k;
  R.dim = G.L.dim;
  R.metric = G.metric;
  const uint32_t d = R.dim;
  const size_t n = sample.size();
  auto row = [&](size_t i) { return &G.vec[static_cast<uint64_t>(sample[i]) * d]; };
  std::mt19937 rng(seed);
  R.centroids.assign(static_cast<size_t>(k) * d, 0.f);
  // k-means++: the first centre uniformly, then proportional to the distance to the nearest chosen centre
  std::vector<float> best(n, std::numeric_limits<float>::max());
  size_t pick = std::uniform_int_distribution<size_t>(0, n - 1)(rng);
  for (uint32_t c = 0; c < k; ++c) {
    std::copy(row(pick), row(pick) + d, &R.centroids[static_cast<size_t>(c) * d]);
    double total = 0;
    for (size_t i = 0; i < n; ++i) {
      const float dd = std::max(0.f, region_dist(0, row(i), &R.centroids[static_cast<size_t>(c) * d], d));
      best[i] = std::min(best[i], dd);
      total += best[i];
    }
    if (total <= 0) break;
    double u = std::uniform_real_distribution<double>(0, total)(rng);
    for (size_t i = 0; i < n; ++i) {
      u -= best[i];
      if (u <= 0) {
        pick = i;
        break;
      }
    }
  }
  std::vector<uint32_t> asg(n, 0);
  for (int iter = 0; iter < 1000; ++iter) {
    for (size_t i = 0; i < n; ++i) asg[i] = nearest_region(R, row(i));
    std::vector<double> sum(static_cast<size_t>(k) * d, 0.0);
    std::vector<size_t> cnt(k, 0);
    for (size_t i = 0; i < n; ++i) {
      ++cnt[asg[i]];
      for (uint32_t j = 0; j < d; ++j) sum[static_cast<size_t>(asg[i]) * d + j] += row(i)[j];
    }
    double moved = 0;
    for (uint32_t c = 0; c < k; ++c) {
      if (!cnt[c]) continue;  // an empty cluster keeps its centre
      double m2 = 0;
      for (uint32_t j = 0; j < d; ++j) {
        const float v = static_cast<float>(sum[static_cast<size_t>(c) * d + j] / cnt[c]);
        const double t = v - R.centroids[static_cast<size_t>(c) * d + j];
        m2 += t * t;
        R.centroids[static_cast<size_t>(c) * d + j] = v;
      }
      moved += std::sqrt(m2);
    }
    if (moved <= 1e-3) break;
  }
  return R;
}

uint32_t nearest_region(const Regions& R, const float* x) {
  uint32_t b = 0;
  float bd = std::numeric_limits<float>::max();
  for (uint32_t c = 0; c < R.k; ++c) {
    const float dd = region_dist(R.metric, x, &R.centroids[static_cast<size_t>(c) * R.dim], R.dim);
    if (dd < bd) {
      bd = dd;
      b = c;
    }
  }
  return b;
}

// Balanced assignment: each item goes to its closest region that is below `limit`, the next closest otherwise
// (query_router.hh:359-372, BALANCED_ROUTING).  Items are taken in `order`.
static void assign_balanced(const Regions& R, const float* xs, uint64_t n, uint64_t stride, uint64_t limit,
                            const std::vector<uint64_t>& order, uint32_t* out) {
  std::vector<uint64_t> fill(R.k, 0);
  std::vector<std::pair<float, uint32_t>> cand(R.k);
  for (uint64_t oi = 0; oi < n; ++oi) {
    const uint64_t i = order[oi];
    const float* x = xs + i * stride;
    for (uint32_t c = 0; c < R.k; ++c)
      cand[c] = {region_dist(R.metric, x, &R.centroids[static_cast<size_t>(c) * R.dim], R.dim), c};
    std::sort(cand.begin(), cand.end());
    uint32_t dest = cand[0].second;
    for (auto& [dd, c] : cand)
      if (fill[c] < limit) {
        dest = c;
        break;
      }
    ++fill[dest];
    out[i] = dest;
  }
}

std::vector<uint32_t> assign_regions(const HostGraph& G, const Regions& R, double slack, uint32_t seed) {
  std::vector<uint32_t> owner(G.N, 0);
  const uint64_t limit = static_cast<uint64_t>(std::ceil(static_cast<double>(G.N) / R.k * (1.0 + slack)));
  std::vector<uint64_t> order(G.N);
  std::iota(order.begin(), order.end(), 0);
  std::shuffle(order.begin(), order.end(), std::mt19937_64(seed));  // no region fills up first by record order
  assign_balanced(R, G.vec.data(), G.N, G.L.dim, limit, order, owner.data());
  return owner;
}

void route_queries(const Regions& R, const float* q, uint32_t nq, double slack, uint32_t* out) {
  const uint64_t limit = std::max<uint64_t>(1, static_cast<uint64_t>(std::ceil(static_cast<double>(nq) / R.k * (1.0 + slack))));
  std::vector<uint64_t> order(nq);
  std::iota(order.begin(), order.end(), 0);  // batch order, as the router thread takes its queue
  assign_balanced(R, q, nq, R.dim, limit, order, out);
}

}  // namespace shine
