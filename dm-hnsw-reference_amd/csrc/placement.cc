// Region placement of a sharded index and query routing: the GPU-node form of the reference's Placement / Kmeans /
// QueryRouter (src/cache/placement.hh:9-111, src/cache/kmeans.hh:10-378, src/router/query_router.hh:18-427).
//
// The reference clusters the top-level nodes with balanced k-means and routes every query to the compute node whose
// centroid is closest, within per-batch limits that adapt to the nodes' queue sizes, so that each node's cache
// serves one region of the space.  Here the k regions are the GPU slots of a sharded index: every record is owned by
// the slot of its region, and a query routed to its region reads mostly that GPU's own HBM.  Host code, run once at
// open and per batch for routing.
//
// Arithmetic follows the reference's types: f32 sums, means, sizes-as-f32 and penalties, f64 limits; distances in
// the order of hostdist.h.  The reference's build adds -ffast-math (CMakeLists.txt:16), which lets the compiler
// contract or reassociate these f32 expressions; this restatement evaluates them as written.
#include "placement.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>

#include "hostdist.h"

namespace shine {

namespace {

constexpr float kFltMax = std::numeric_limits<float>::max();

inline float kdist(const KmeansInput& in, const float* a, const float* b) { return host_dist(in.metric, a, b, in.dim); }

// init_plusplus (kmeans.hh:163-197): the first centre drawn uniformly with std::mt19937{1234}, then repeatedly the
// row whose closest chosen centre is farthest (the first maximum), over the chosen rows themselves
std::vector<float> init_plusplus(const KmeansInput& in, uint32_t k) {
  const size_t n = in.rows.size(), d = in.dim;
  std::vector<size_t> chosen;
  chosen.reserve(k);
  {
    std::mt19937 generator{1234};
    std::uniform_int_distribution<size_t> pick(0, n - 1);
    chosen.push_back(pick(generator));
  }
  std::vector<float> closest(n);
  while (chosen.size() < k) {
    for (size_t i = 0; i < n; ++i) {  // closest_distances (kmeans.hh:143-161)
      float c = kFltMax;
      for (const size_t j : chosen) {
        const float t = kdist(in, in.rows[i], in.rows[j]);
        if (t < c) c = t;
      }
      closest[i] = c;
    }
    chosen.push_back(static_cast<size_t>(std::max_element(closest.begin(), closest.end()) - closest.begin()));
  }
  std::vector<float> centroids(static_cast<size_t>(k) * d);
  for (uint32_t c = 0; c < k; ++c) std::copy(in.rows[chosen[c]], in.rows[chosen[c]] + d, &centroids[c * d]);
  return centroids;
}

// compute_cluster_assignment (kmeans.hh:202-223): the first closest centroid
uint32_t closest_centroid(const KmeansInput& in, const float* x, const std::vector<float>& centroids, uint32_t k) {
  float best = kFltMax;
  uint32_t index = 0;
  for (uint32_t c = 0; c < k; ++c) {
    const float t = kdist(in, x, &centroids[static_cast<size_t>(c) * in.dim]);
    if (t < best) {
      best = t;
      index = c;
    }
  }
  return index;
}

std::vector<uint32_t> assign(const KmeansInput& in, const std::vector<float>& centroids, uint32_t k) {
  std::vector<uint32_t> a(in.rows.size());
  for (size_t i = 0; i < in.rows.size(); ++i) a[i] = closest_centroid(in, in.rows[i], centroids, k);
  return a;
}

// calculate_means (kmeans.hh:225-252): f32 sums in row order; an empty cluster keeps its old centroid
std::vector<float> calculate_means(const KmeansInput& in, const std::vector<uint32_t>& asg,
                                   const std::vector<float>& old, uint32_t k) {
  const size_t d = in.dim;
  std::vector<float> c(static_cast<size_t>(k) * d, 0.f);
  std::vector<float> count(k, 0.f);
  for (size_t i = 0; i < in.rows.size(); ++i) {
    float* nc = &c[asg[i] * d];
    ++count[asg[i]];
    for (size_t j = 0; j < d; ++j) nc[j] += in.rows[i][j];
  }
  for (uint32_t i = 0; i < k; ++i) {
    if (count[i] == 0) {
      std::copy(&old[i * d], &old[i * d] + d, &c[i * d]);
    } else {
      for (size_t j = 0; j < d; ++j) c[i * d + j] /= count[i];
    }
  }
  return c;
}

}  // namespace

KmeansResult run_kmeans(const KmeansInput& in, uint32_t k) {
  KmeansResult r;
  const size_t d = in.dim;
  float error = kFltMax;
  uint32_t iteration = 0;
  while (iteration < kKmeansIterationLimit && error > 0.001) {
    std::vector<float> nc = iteration == 0 ? init_plusplus(in, k) : calculate_means(in, r.assignment, r.centroids, k);
    r.assignment = assign(in, nc, k);
    if (iteration > 0) {  // total movement of the centroids: Σ sqrt(L2), or Σ IP distance (kmeans.hh:108-118)
      error = 0.f;
      for (uint32_t i = 0; i < k; ++i) {
        const float t = kdist(in, &r.centroids[i * d], &nc[i * d]);
        error += in.metric == 0 ? std::sqrt(t) : t;
      }
    }
    r.centroids = std::move(nc);
    ++iteration;
  }
  r.sizes.assign(k, 0);
  for (const uint32_t a : r.assignment) ++r.sizes[a];
  r.iterations = iteration;
  r.error = error;
  return r;
}

// Algorithm 1 of "Balanced k-means revisited" as kmeans.hh:259-377 states it: every row in turn leaves its cluster
// (whose centroid is updated without it) and joins the cluster of least cost dist + p_now * size among those the
// current penalty allows; p_next, the smallest penalty that would allow one more move, raises p_now after each pass.
std::vector<uint64_t> balanced_kmeans(const KmeansInput& in, uint32_t k, float c, float penalty_factor,
                                      uint32_t max_cluster_size_difference, KmeansResult& r, uint32_t* iterations) {
  const size_t n = in.rows.size(), d = in.dim;
  std::vector<float>& centroids = r.centroids;
  std::vector<uint32_t>& asg = r.assignment;
  std::vector<uint64_t>& sizes = r.sizes;
  float p_now = 0.f, p_next = kFltMax;
  uint64_t n_min = 0, n_max = n;
  uint32_t iter = 0;
  std::vector<float> sum(static_cast<size_t>(k) * d, 0.f);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < d; ++j) sum[asg[i] * d + j] += in.rows[i][j];

  while (n_max - n_min > max_cluster_size_difference && iter < kKmeansIterationLimit) {
    for (size_t ni = 0; ni < n; ++ni) {
      const float* x = in.rows[ni];
      const uint32_t old = asg[ni];
      if (sizes[old] == 1) continue;  // a cluster never empties
      float* oc = &centroids[old * d];
      for (size_t j = 0; j < d; ++j) {
        sum[old * d + j] -= x[j];
        oc[j] = sum[old * d + j] / static_cast<float>(sizes[old] - 1);
      }
      --sizes[old];
      uint32_t& dest = asg[ni];
      float cost = kFltMax;
      const float dist_old = kdist(in, oc, x);
      const float old_size = static_cast<float>(sizes[old]) + c;
      for (uint32_t j = 0; j < k; ++j) {
        const float dist_j = kdist(in, &centroids[j * d], x);
        const float size_j = static_cast<float>(sizes[j]);
        const float needed = (dist_j - dist_old) / (old_size - size_j);
        if (old_size > size_j) {  // a smaller cluster: joined once the penalty reaches `needed`
          if (p_now < needed) {
            if (needed < p_next) p_next = needed;
          } else if (dist_j + p_now * size_j < cost && j != old) {
            cost = dist_j + p_now * size_j;
            dest = j;
          }
        } else if (p_now < needed && dist_j + p_now * size_j < cost) {  // a larger one: while it is still worth it
          cost = dist_j + p_now * size_j;
          dest = j;
        }
      }
      float* nc = &centroids[dest * d];
      for (size_t j = 0; j < d; ++j) {
        sum[dest * d + j] += x[j];
        nc[j] = sum[dest * d + j] / static_cast<float>(sizes[dest] + 1);
      }
      ++sizes[dest];
    }
    n_min = *std::min_element(sizes.begin(), sizes.end());
    n_max = *std::max_element(sizes.begin(), sizes.end());
    p_now = penalty_factor * p_next;
    p_next = kFltMax;
    ++iter;
  }
  if (iterations) *iterations = iter;
  std::vector<uint64_t> actual(k, 0);  // sizes of the nearest-centroid partition (kmeans.hh:356-369)
  for (size_t i = 0; i < n; ++i) ++actual[closest_centroid(in, in.rows[i], centroids, k)];
  return actual;
}

int run_and_optimize(const KmeansInput& in, uint32_t k, bool balanced, Regions& out) {
  out = Regions{};
  out.k = k;
  out.dim = in.dim;
  out.metric = in.metric;
  if (k == 0) return -1;
  if (!balanced) {  // Placement's plain branch: run_kmeans with k clusters, identity mapping (placement.hh:45-58)
    if (in.rows.size() < k) return -1;
    KmeansResult r = run_kmeans(in, k);
    out.centroids = std::move(r.centroids);
    out.mapping.resize(k);
    std::iota(out.mapping.begin(), out.mapping.end(), 0u);
    out.sizes = r.sizes;
    out.iterations = r.iterations;
    return 0;
  }
  const uint32_t local_k = k % 2 == 0 ? k : 2 * k;  // odd k: 2k clusters, merged in pairs below
  if (in.rows.size() < local_k) return -1;
  KmeansResult r = run_kmeans(in, local_k);
  out.iterations = r.iterations;
  const std::vector<uint64_t> bal = balanced_kmeans(in, local_k, 0.15f, 1.01f, 1, r, &out.balance_iterations);
  out.centroids = r.centroids;
  out.mapping.assign(local_k, 0);
  out.sizes.assign(k, 0);
  if (k % 2 == 0) {
    std::iota(out.mapping.begin(), out.mapping.end(), 0u);
    out.sizes = bal;
    return 0;
  }
  // each cluster not yet paired takes its closest unpaired successor (kmeans.hh:46-77)
  std::vector<bool> paired(local_k, false);
  const size_t d = in.dim;
  for (uint32_t i = 0, next = 0; i < local_k; ++i) {
    if (paired[i]) continue;
    float min_dist = kFltMax;
    uint32_t min_pos = 0;
    for (uint32_t j = i + 1; j < local_k; ++j) {
      if (paired[j]) continue;
      const float t = kdist(in, &out.centroids[i * d], &out.centroids[j * d]);
      if (t < min_dist) {
        min_dist = t;
        min_pos = j;
      }
    }
    if (min_pos == i) return -1;  // lib_assert(i != min_pos, "invalid assignment")
    paired[i] = paired[min_pos] = true;
    out.mapping[i] = out.mapping[min_pos] = next;
    out.sizes[next] = bal[i] + bal[min_pos];
    ++next;
  }
  return 0;
}

// Breadth-first over the lists of the top level from the entry point, one level lower while fewer than min_nodes
// were found.  Every node reached at level l has a list at level l (it came from a list at a level >= l).
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

int plan_regions(const HostGraph& G, uint32_t k, bool balanced, Regions& out) {
  const std::vector<uint32_t> sample = top_level_sample(G, kFetchLevelNodes);
  KmeansInput in;
  in.metric = G.metric;
  in.dim = G.L.dim;
  in.rows.reserve(sample.size());
  for (const uint32_t s : sample) in.rows.push_back(&G.vec[static_cast<uint64_t>(s) * G.L.dim]);
  return run_and_optimize(in, k, balanced, out);
}

// MinPlacement is heap::Heap<pair<idx_t, distance_t>, MinHeapPlacementCompare>: std::push_heap of every
// (mapping[i], distance) in centroid order, then std::pop_heap until empty
void closest_regions(const Regions& R, const float* x, std::vector<uint32_t>& order) {
  using Entry = std::pair<size_t, float>;
  const auto cmp = [](const Entry& l, const Entry& r) { return l.second > r.second; };
  std::vector<Entry> heap;
  heap.reserve(R.n_centroids());
  for (uint32_t i = 0; i < R.n_centroids(); ++i) {
    heap.emplace_back(R.mapping[i], host_dist(R.metric, x, &R.centroids[static_cast<size_t>(i) * R.dim], R.dim));
    std::push_heap(heap.begin(), heap.end(), cmp);
  }
  order.clear();
  while (!heap.empty()) {
    order.push_back(static_cast<uint32_t>(heap.front().first));
    std::pop_heap(heap.begin(), heap.end(), cmp);
    heap.pop_back();
  }
}

uint32_t nearest_region(const Regions& R, const float* x) {
  std::vector<uint32_t> order;
  closest_regions(R, x, order);
  return order.empty() ? 0 : order.front();
}

std::vector<uint32_t> assign_regions(const HostGraph& G, const Regions& R, double slack, uint32_t seed) {
  std::vector<uint32_t> owner(G.N, 0);
  const uint64_t limit = static_cast<uint64_t>(std::ceil(static_cast<double>(G.N) / R.k * (1.0 + slack)));
  std::vector<uint64_t> order(G.N);
  std::iota(order.begin(), order.end(), 0);
  std::shuffle(order.begin(), order.end(), std::mt19937_64(seed));  // no region fills up first by record order
  std::vector<uint64_t> fill(R.k, 0);
  std::vector<uint32_t> cand;
  for (const uint64_t i : order) {
    closest_regions(R, &G.vec[i * G.L.dim], cand);
    uint32_t dest = 0;
    for (const uint32_t c : cand) {  // as the router: the first with room, else the last one popped
      dest = c;
      if (fill[c] < limit) break;
    }
    ++fill[dest];
    owner[i] = dest;
  }
  return owner;
}

void Router::init(uint32_t regions) {
  k = regions;
  batch_size = static_cast<uint64_t>(kLimitPerCn) * k;
  local_slot = 0;
  limits.assign(k, kLimitPerCn);
  histogram.assign(k, 0);
}

// update_limits (query_router.hh:106-151): a node's share of the next batch grows as its queue shrinks relative to
// the others', scale_i = (Σp - p_i) / Σ_j(Σp - p_j) * k, truncated, then topped up round robin to batch_size
bool Router::update_limits(const std::vector<uint32_t>& progresses) {
  const double sum = static_cast<double>(std::accumulate(progresses.begin(), progresses.end(), 0u));
  if (sum < k || k < 2) return false;  // k = 1: the reference's denominator is 0 (one node routes to itself)
  double denom = 0;
  for (uint32_t i = 0; i < k; ++i) denom += sum - progresses[i];
  uint64_t total = 0;
  for (uint32_t i = 0; i < k; ++i) {
    const double scale = ((sum - progresses[i]) / denom) * static_cast<double>(k);
    limits[i] = static_cast<uint64_t>(static_cast<double>(kLimitPerCn) * scale);
    total += limits[i];
  }
  for (uint64_t i = 0; total < batch_size; ++i) {
    ++limits[i % k];
    ++total;
  }
  return true;
}

void Router::route(const Regions& R, const float* q, uint32_t nq, uint64_t stride,
                   const std::function<void(const std::vector<uint64_t>&, std::vector<uint32_t>&)>& progress,
                   uint32_t* out) {
  std::vector<uint64_t> routed(k, 0);
  std::vector<uint32_t> prog(k, 0), order;
  for (uint32_t i = 0; i < nq; ++i) {
    if (local_slot > 0 && local_slot % batch_size == 0) {  // a batch is done: sync point (query_router.hh:299-324)
      std::fill(histogram.begin(), histogram.end(), 0);
      if (adaptive) {
        std::fill(prog.begin(), prog.end(), 0);
        if (progress) progress(routed, prog);
        update_limits(prog);
      }
    }
    closest_regions(R, q + static_cast<uint64_t>(i) * stride, order);
    uint32_t dest = 0;
    for (const uint32_t c : order) {  // BALANCED_ROUTING (query_router.hh:355-368)
      dest = c;
      if (histogram[dest] < limits[dest]) break;
    }
    ++histogram[dest];
    ++routed[dest];
    out[i] = dest;
    ++local_slot;
  }
}

}  // namespace shine
