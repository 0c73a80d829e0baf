// SPDX-License-Identifier: MIT
//
// ============================================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product path.
//  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, as the checker.
// ============================================================================================================
//
//  A CPU restatement of the SHINE compute-node query path and of the insert path that produces the index it
//  reads.  Every function cites the reference file:line it follows (paths relative to the reference repo root).
//  The restatement keeps the reference's own C++ standard-library calls where they decide results:
//    * heaps: std::push_heap / std::pop_heap / std::make_heap with the reference comparators (src/hnsw/heap.hh)
//    * sort:  std::sort with the (distance, id) tie-break                                   (src/hnsw/heap.hh:53-57)
//    * level draw: std::mt19937 + std::uniform_real_distribution<double>                    (src/hnsw/hnsw.hh:34-48)
//  so the third-party arithmetic on the path (libstdc++, g++ 11.4 here; the reference pins g++-12, README.md:19)
//  is executed, not re-implemented.  What is dropped: RDMA verbs, coroutines, shared_ptr node copies, the
//  compute-node cache (hit/miss does not change results), routing.
//
//  Distance FP order.  The reference computes L2 / IP with hnswlib's AVX2 kernels under -O3 -march=native
//  -ffast-math (src/hnsw/distance.hh:11-151, CMakeLists.txt:16), so their rounding is whatever GCC makes of the
//  expressions, and that is not one fixed order: `l2_as_written` / `ip_as_written` below restate the expressions
//  with no order pinned, and GCC 11.4 -ffast-math reassociates them (per 16-wide block t = fma(x0, y0, rn(x1*y1)),
//  acc += t; the eight lanes summed as a tree whose pairing changes with the inlining context, e.g.
//  ((t0+t1)+(t2+t3))+((t4+t5)+(t6+t7)) inlined, ((t3+t4)+(t5+t7))+((t0+t2)+(t1+t6)) out of line; IP's
//  `1 - (sum + tail)` distributed into a chain of subtractions).  The reference's own call sites (inlined into
//  search_for_one / search_level) may each round differently, so no restatement can reproduce its float roundings
//  bit for bit (tests/test_fp_order.py).  This restatement therefore FIXES one order — 8 lane
//  accumulators, lane j an fma chain over elements i ≡ j (mod 8) of the 16-aligned prefix, the lanes added left to
//  right, then the scalar tail — compiled with -ffp-contract=off + explicit fmaf / _mm256_fmadd_ps so the order is
//  exactly what is written; the GPU kernels and the builder use the same order.  The reference-flags build
//  (`make native`, bench.py's CPU baseline) evaluates the as-written form instead, as the reference's build does.
//  On integer-valued data (SIFT-like) every partial sum is exact (< 2^24) and all of these agree bit for bit.
//
//  Parity status: the reference ships no tests, fixtures or golden vectors, and compiling/running it in this
//  pipeline was refused.  The heap / sort / RNG behaviour is pinned against libstdc++ itself
//  (tests/test_oracle.py runs oracle_selftest_*), the rest is PARITY UNPINNED by any reference output.
// ============================================================================================================

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>

#include <pthread.h>
#include <sched.h>
#include <unordered_set>
#include <vector>

#if defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
#define ORACLE_AVX2 1
#endif

namespace oracle {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using f32 = float;
using f64 = double;

// ---------------------------------------------------------------------------------------------------------
// distance.hh:11-161
// ---------------------------------------------------------------------------------------------------------
static inline f32 hsum8_ltr(const f32* t) {  // TmpRes[0] + ... + TmpRes[7], left to right (distance.hh:40)
  f32 s = t[0];
  for (int j = 1; j < 8; ++j) s = s + t[j];
  return s;
}

// l2 (distance.hh:80-118) -> L2SqrSIMD16ExtAVX (distance.hh:11-41) on the first dim>>4<<4 elements + scalar tail
static f32 l2(const f32* a, const f32* b, size_t dim) {
  const size_t q16 = dim >> 4 << 4;
  alignas(32) f32 acc[8];
#ifdef ORACLE_AVX2
  __m256 sum = _mm256_setzero_ps();
  for (size_t i = 0; i < q16; i += 8) {
    const __m256 d = _mm256_sub_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i));
    sum = _mm256_fmadd_ps(d, d, sum);
  }
  _mm256_store_ps(acc, sum);
#else
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (size_t i = 0; i < q16; i += 8)
    for (int j = 0; j < 8; ++j) {
      const f32 d = a[i + j] - b[i + j];
      acc[j] = std::fmaf(d, d, acc[j]);
    }
#endif
  f32 result = hsum8_ltr(acc);
  for (size_t i = q16; i < dim; ++i) {  // distance.hh:112-115 (result += diff0 * diff0, contracted)
    const f32 d = a[i] - b[i];
    result = std::fmaf(d, d, result);
  }
  return result;
}

// ip_distance (distance.hh:120-151) -> InnerProductSIMD16ExtAVX (distance.hh:44-76) + tail; result = 1 - dot
static f32 ip_distance(const f32* a, const f32* b, size_t dim) {
  const size_t q16 = dim >> 4 << 4;
  alignas(32) f32 acc[8];
#ifdef ORACLE_AVX2
  __m256 sum = _mm256_setzero_ps();
  for (size_t i = 0; i < q16; i += 8) sum = _mm256_fmadd_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i), sum);
  _mm256_store_ps(acc, sum);
#else
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (size_t i = 0; i < q16; i += 8)
    for (int j = 0; j < 8; ++j) acc[j] = std::fmaf(a[i + j], b[i + j], acc[j]);
#endif
  const f32 res = hsum8_ltr(acc);
  f32 res_tail = 0.f;
  for (size_t i = q16; i < dim; ++i) res_tail = std::fmaf(a[i], b[i], res_tail);  // distance.hh:136-139
  return 1.0f - (res + res_tail);                                                  // distance.hh:141
}

// ---- The same two distances in the reference's expression shape (distance.hh:11-76, 80-151), with no FP order
// pinned: per 16-wide step two 8-lane updates `acc = acc + d * d` (`acc + a * b`), the eight lanes summed in one
// expression, then the scalar tail as a running `+=`.  How these round is left to the compiler: under the
// reference's flags (-O3 -march=native -ffast-math -mavx2, CMakeLists.txt:16) GCC contracts and reassociates
// them.  The native (reference-flags) build of the oracle evaluates these, the CPU baseline times them, and
// tests/test_fp_order.py checks that the fixed-order functions above reproduce them bit for bit.
#ifdef ORACLE_AVX2
static f32 l2_as_written(const f32* a, const f32* b, size_t dim) {
  const size_t q16 = dim >> 4 << 4;
  __m256 acc = _mm256_setzero_ps();
  for (size_t i = 0; i < q16; i += 16) {
    __m256 d = _mm256_sub_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i));
    acc = _mm256_add_ps(acc, _mm256_mul_ps(d, d));
    d = _mm256_sub_ps(_mm256_loadu_ps(a + i + 8), _mm256_loadu_ps(b + i + 8));
    acc = _mm256_add_ps(acc, _mm256_mul_ps(d, d));
  }
  alignas(32) f32 t[8];
  _mm256_store_ps(t, acc);
  f32 r = t[0] + t[1] + t[2] + t[3] + t[4] + t[5] + t[6] + t[7];
  for (size_t i = q16; i < dim; ++i) {
    const f32 d = a[i] - b[i];
    r += d * d;
  }
  return r;
}

static f32 ip_as_written(const f32* a, const f32* b, size_t dim) {
  const size_t q16 = dim >> 4 << 4;
  __m256 acc = _mm256_setzero_ps();
  for (size_t i = 0; i < q16; i += 16) {
    acc = _mm256_add_ps(acc, _mm256_mul_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i)));
    acc = _mm256_add_ps(acc, _mm256_mul_ps(_mm256_loadu_ps(a + i + 8), _mm256_loadu_ps(b + i + 8)));
  }
  alignas(32) f32 t[8];
  _mm256_store_ps(t, acc);
  const f32 r = t[0] + t[1] + t[2] + t[3] + t[4] + t[5] + t[6] + t[7];
  f32 tail = 0;
  for (size_t i = q16; i < dim; ++i) tail += a[i] * b[i];
  return 1.0f - (r + tail);
}
#endif

// L2Distance / IPDistance (distance.hh:153-161).  The reference-flags build (CPU baseline) evaluates the
// as-written form, as the reference's own build does; the checker evaluates the fixed order.
static inline f32 distance(int metric, const f32* a, const f32* b, size_t dim) {
#if defined(__FAST_MATH__) && defined(ORACLE_AVX2)
  return metric == 1 ? ip_as_written(a, b, dim) : l2_as_written(a, b, dim);
#else
  return metric == 1 ? ip_distance(a, b, dim) : l2(a, b, dim);
#endif
}

// ---------------------------------------------------------------------------------------------------------
// remote_pointer.hh:7-29 — [memory node (16b) | byte offset (48b)]
// ---------------------------------------------------------------------------------------------------------
static inline u32 rp_node(u64 r) { return static_cast<u32>(r >> 48); }
static inline u64 rp_off(u64 r) { return (r << 16) >> 16; }
static inline u64 rp_make(u32 node, u64 off) { return (static_cast<u64>(node) << 48) | off; }

// ---------------------------------------------------------------------------------------------------------
// node.hh:10-54 / node.cc:18-27 — record layout
//   hdr u64 | uid u32 | level u32 | d×f32 | L0: cnt u32 + 2M×u64 | L≥1: cnt u32 + M×u64 (each level)
// ---------------------------------------------------------------------------------------------------------
constexpr u64 HEADER_NODE_LOCK = 0b01;                 // node.hh:28
constexpr u64 HEADER_NEW_LEVEL_LOCK = 0b100000000;     // node.hh:29
constexpr u64 HEADER_ENTRY_NODE = 0b10000000000000000; // node.hh:30

struct Layout {
  u32 dim = 0, m = 0, m_max = 0, m_max_zero = 0;
  size_t nl_zero = 0, nl = 0;  // NEIGHBORLIST_SIZE_ZERO / NEIGHBORLIST_SIZE (node.hh:44-48)
  void init(u32 d, u32 M) {
    dim = d; m = M; m_max = M; m_max_zero = 2 * M;  // hnsw.hh:26-28
    nl_zero = sizeof(u32) + m_max_zero * sizeof(u64);
    nl = sizeof(u32) + m_max * sizeof(u64);
  }
  size_t size_until_components() const { return 16 + dim * sizeof(f32); }  // node.hh:50
  size_t total_size(u32 level) const { return size_until_components() + nl_zero + level * nl; }  // node.hh:51-54
  size_t alloc_size(u32 level) const {  // rdma_atomics.hh:90-95 (pad with 4-byte steps to 8 B)
    size_t s = total_size(level);
    while (s % 8 != 0) s += 4;
    return s;
  }
  size_t list_offset(u64 node_off, u32 lvl) const {  // node.cc:18-27
    size_t o = node_off + size_until_components();
    if (lvl > 0) o += nl_zero + (lvl - 1) * nl;
    return o;
  }
};

struct Entry {  // heap.hh:10-13 (s_ptr<Node> replaced by the node's RemotePtr)
  u64 node;
  f32 distance;
};
struct MaxHeapCompare {  // heap.hh:15-17
  bool operator()(const Entry& l, const Entry& r) const { return l.distance < r.distance; }
};
struct MinHeapCompare {  // heap.hh:19-21
  bool operator()(const Entry& l, const Entry& r) const { return l.distance > r.distance; }
};

template <class Compare>
struct Heap {  // heap.hh:23-62
  std::vector<Entry> heap;
  void make_heap() { std::make_heap(heap.begin(), heap.end(), Compare()); }
  void clear() { heap.clear(); }
  void push_k(const Entry& e, size_t k) {  // heap.hh:34-41
    if (size() < k) {
      push(e);
    } else if (Compare()(e, top())) {
      pop();
      push(e);
    }
  }
  void push(const Entry& e) {  // heap.hh:43-46
    heap.push_back(e);
    std::push_heap(heap.begin(), heap.end(), Compare());
  }
  void pop() {  // heap.hh:48-51
    std::pop_heap(heap.begin(), heap.end(), Compare());
    heap.pop_back();
  }
  template <class IdOf>
  void sort_ascending(IdOf id_of) {  // heap.hh:53-57 — ties broken by node id
    std::sort(heap.begin(), heap.end(), [&](const Entry& l, const Entry& r) {
      return l.distance == r.distance ? id_of(l.node) < id_of(r.node) : l.distance < r.distance;
    });
  }
  Entry top() const { return heap.front(); }
  size_t size() const { return heap.size(); }
  bool empty() const { return heap.empty(); }
};
using MaxHeap = Heap<MaxHeapCompare>;  // heap.hh:65
using MinHeap = Heap<MinHeapCompare>;  // heap.hh:66

// Per-query counters: the subset of statistics.hh:148-175 the query path touches, plus the split by level
// that the roofline needs.  Layout is shared with the GPU path (include/shine_gpu.h, SHINE_QS_*).
enum : int {
  QS_DISTCOMPS = 0,
  QS_VISITED_UPPER = 1,   // stats.visited_nodes        (statistics.hh:155, inc_visited_nodes level>0)
  QS_VISITED_L0 = 2,      // stats.visited_nodes_l0     (statistics.hh:156)
  QS_LISTS_UPPER = 3,     // stats.visited_neighborlists at level > 0  (hnsw.hh:359)
  QS_LISTS_L0 = 4,        // stats.visited_neighborlists at level 0    (hnsw.hh:438)
  QS_MAX_NEXT = 5,        // diagnostic: peak size of next_candidates
  QS_STATUS = 6,
  QS_NRESULT = 7,
  QS_WORDS = 8
};

struct Index {
  Layout L;
  int metric = 0;  // 0 = squared L2, 1 = inner product (main.cc:15-21 --ip-dist)
  std::vector<std::vector<u8>> shards;  // memory_node.hh:15-27: [free_ptr | ep_ptr | records...]
  // build-only state
  u64 build_distcomps = 0;
  u32 max_level = 0;

  const u8* at(u64 r) const { return shards[rp_node(r)].data() + rp_off(r); }
  u8* at_mut(u64 r) { return shards[rp_node(r)].data() + rp_off(r); }
  u64 header(u64 r) const { u64 h; std::memcpy(&h, at(r), 8); return h; }
  void set_header(u64 r, u64 h) { std::memcpy(at_mut(r), &h, 8); }
  u32 uid(u64 r) const { u32 v; std::memcpy(&v, at(r) + 8, 4); return v; }     // node.hh:86
  u32 level(u64 r) const { u32 v; std::memcpy(&v, at(r) + 12, 4); return v; }  // node.hh:87
  const f32* comps(u64 r) const { return reinterpret_cast<const f32*>(at(r) + 16); }  // node.hh:90-92
  u64 ep_ptr() const { u64 v; std::memcpy(&v, shards[0].data() + 8, 8); return v; }  // rdma_reads.hh:74-99
  void set_ep_ptr(u64 v) { std::memcpy(shards[0].data() + 8, &v, 8); }  // rdma_writes.hh:198-213
  // neighbour list of node r at level lvl (neighborlist.hh:27-38); read whole (rdma_reads.hh:40-72)
  const u8* list(u64 r, u32 lvl) const {
    return shards[rp_node(r)].data() + L.list_offset(rp_off(r), lvl);
  }
  u8* list_mut(u64 r, u32 lvl) { return shards[rp_node(r)].data() + L.list_offset(rp_off(r), lvl); }
  static u32 list_count(const u8* l) { u32 c; std::memcpy(&c, l, 4); return c; }
  static u64 list_at(const u8* l, u32 i) { u64 v; std::memcpy(&v, l + 4 + 8 * i, 8); return v; }
  f32 dist(const f32* a, const f32* b) const { return distance(metric, a, b, L.dim); }
};

// ---------------------------------------------------------------------------------------------------------
// Per-coroutine search state (coroutine.hh:58-62) and the query/insert algorithms (hnsw.hh)
// ---------------------------------------------------------------------------------------------------------
struct SearchState {
  std::unordered_set<u64> visited_nodes;  // hashset_t<RemotePtr> (types.hh:14-15)
  MaxHeap top_candidates;
  MinHeap next_candidates;
  u32 qs[QS_WORDS] = {0};
  u64 distcomps = 0;
  // record reads in order (nullable): every cache_lookup of a node (hnsw.hh:263, 368, 449), as (node, admit-always)
  std::vector<std::pair<u64, bool>>* reads = nullptr;
  void read(u64 r, bool always) {
    if (reads) reads->emplace_back(r, always);
  }
};

// hnsw.hh:331-393 — greedy 1-NN descent from begin_level down to target_level+1
static void search_for_one(const Index& I, const f32* q, u64& nearest_neighbor, f32 closest_distance,
                           u32 begin_level, u32 target_level, SearchState& st) {
  bool changed;
  for (u32 level = begin_level; level > target_level; level--) {
    do {
      changed = false;
      const u8* nl = I.list(nearest_neighbor, level);  // :356-358
      ++st.qs[QS_LISTS_UPPER];
      u64 best_candidate = 0;
      const u32 cnt = Index::list_count(nl);
      for (u32 i = 0; i < cnt; ++i) {  // :364
        const u64 r_ptr = Index::list_at(nl, i);
        st.read(r_ptr, true);       // cache_lookup, inner nodes always admitted (:368)
        ++st.qs[QS_VISITED_UPPER];  // inc_visited_nodes(level), level > 0
        const f32 d = I.dist(q, I.comps(r_ptr));  // :375
        ++st.distcomps;
        if (d < closest_distance) {  // :378 strict
          closest_distance = d;
          best_candidate = r_ptr;
          changed = true;
        }
      }
      nearest_neighbor = changed ? best_candidate : nearest_neighbor;  // :385
    } while (changed);
  }
}

// hnsw.hh:406-476 — best-first beam search on one level; top_candidates holds the entry point(s) on entry
static void search_level(const Index& I, const f32* q, u32 ef, u32 level, SearchState& st) {
  auto& visited = st.visited_nodes;
  auto& top = st.top_candidates;
  auto& next = st.next_candidates;
  for (const auto& e : top.heap) {  // :412-415
    next.push(e);
    visited.insert(e.node);
  }
  u32 max_next = static_cast<u32>(next.size());
  while (!next.empty()) {  // :417
    const Entry c = next.top();  // :418-419
    next.pop();
    f32 farthest_dist = top.top().distance;  // :421
    if (c.distance > farthest_dist) break;   // :424 strict
    const u8* nl = I.list(c.node, level);    // :436-437
    if (level > 0) ++st.qs[QS_LISTS_UPPER]; else ++st.qs[QS_LISTS_L0];
    const u32 cnt = Index::list_count(nl);
    for (u32 i = 0; i < cnt; ++i) {  // :440
      const u64 nb = Index::list_at(nl, i);
      if (!visited.contains(nb)) {  // :441
        if (level > 0) ++st.qs[QS_VISITED_UPPER]; else ++st.qs[QS_VISITED_L0];  // :442
        visited.insert(nb);                                                     // :443
        st.read(nb, level > 0);                                                 // cache_lookup (:447-449)
        farthest_dist = top.top().distance;                                     // :456
        const f32 nd = I.dist(q, I.comps(nb));                                   // :458
        ++st.distcomps;
        if (nd < farthest_dist || top.size() < ef) {  // :461
          next.push({nb, nd});                        // :463
          top.push_k({nb, nd}, ef);                   // :464
          if (next.size() > max_next) max_next = static_cast<u32>(next.size());
        }
      }
    }
  }
  if (max_next > st.qs[QS_MAX_NEXT]) st.qs[QS_MAX_NEXT] = max_next;
  next.clear();     // :474
  visited.clear();  // :475
}

// hnsw.hh:253-307 — one query; results are node ids in heap-array order (:300-303)
static void knn(const Index& I, const f32* q, u32 k, u32 ef, SearchState& st, u32* out_ids, f32* out_dists) {
  for (auto& w : st.qs) w = 0;
  st.distcomps = 0;
  const u64 ep_ptr = I.ep_ptr();  // :256-259
  const u64 entry_point = ep_ptr; // cache_lookup → read_node (:261-268)
  st.read(entry_point, true);
  if (I.level(entry_point) > 0) ++st.qs[QS_VISITED_UPPER]; else ++st.qs[QS_VISITED_L0];  // :270
  const f32 ep_distance = I.dist(q, I.comps(entry_point));  // :271
  ++st.distcomps;
  auto& top = st.top_candidates;
  {
    u64 nn = entry_point;
    search_for_one(I, q, nn, ep_distance, I.level(entry_point), 0, st);  // :279
    top.push({nn, I.dist(q, I.comps(nn))});                           // :285
    ++st.distcomps;
  }
  search_level(I, q, ef, 0, st);  // :290
  while (top.size() > k) top.pop();  // :296-298
  u32 n = 0;
  for (const auto& e : top.heap) {  // :300-303
    out_ids[n] = I.uid(e.node);
    if (out_dists) out_dists[n] = e.distance;
    ++n;
  }
  for (u32 i = n; i < k; ++i) {
    out_ids[i] = 0xFFFFFFFFu;
    if (out_dists) out_dists[i] = 0.f;
  }
  st.qs[QS_NRESULT] = n;
  st.qs[QS_DISTCOMPS] = static_cast<u32>(st.distcomps);
  top.clear();  // :305
}

// hnsw.hh:482-522 — neighbour-selection heuristic (build path)
static void select_heuristic(Index& I, MaxHeap& top, u32 m) {
  if (top.size() < m) return;  // :483
  top.sort_ascending([&](u64 r) { return I.uid(r); });  // :488
  const size_t initial = top.size();
  size_t selected = 1, consumed = 1;
  while (selected < m && consumed < initial) {  // :495
    bool is_selected = true;
    const Entry c = top.heap[consumed];
    for (size_t i = 0; i < selected; ++i) {  // :501
      const f32 d = I.dist(I.comps(top.heap[i].node), I.comps(c.node));  // :503
      ++I.build_distcomps;
      if (d < c.distance) { is_selected = false; break; }  // :506
    }
    if (is_selected) {
      std::swap(top.heap[selected], top.heap[consumed]);  // :513
      ++selected;
    }
    ++consumed;
  }
  top.heap.resize(selected);  // :520
  top.make_heap();            // :521
}

// Single-threaded, single-coroutine build (compute thread 0, coroutine 0).  The reference interleaves
// `--coroutines` inserts per thread and T threads; with T = C = 1 its insert order is the slot order.
struct Builder {
  Index& I;
  u32 efc;
  SearchState st;
  u64 cached_ep_ptr = 0;  // coroutine.hh:56
  std::vector<u64> free_ptr;

  Builder(Index& idx, u32 ef_construction) : I(idx), efc(ef_construction) {}

  // rdma_atomics.hh:88-130 — FAA bump allocation on memory node `shard`
  u64 allocate_node(u32 level, u32 shard) {
    const size_t sz = I.L.alloc_size(level);
    const u64 off = free_ptr[shard];
    free_ptr[shard] += sz;
    std::memcpy(I.shards[shard].data(), &free_ptr[shard], 8);
    return rp_make(shard, off);
  }
  // rdma_writes.hh:75-124 + node_utils.hh:17-25 — header | uid | level | components (lists untouched)
  void write_node(u64 r, u32 id, const f32* comps, u32 level, u64 header) {
    u8* p = I.at_mut(r);
    std::memcpy(p, &header, 8);
    std::memcpy(p + 8, &id, 4);
    std::memcpy(p + 12, &level, 4);
    std::memcpy(p + 16, comps, I.L.dim * sizeof(f32));
  }
  // rdma_writes.hh:151-171 — writes count + the used entries only
  void write_list(u64 r, u32 lvl, const std::vector<u64>& entries) {
    u8* l = I.list_mut(r, lvl);
    const u32 c = static_cast<u32>(entries.size());
    std::memcpy(l, &c, 4);
    for (u32 i = 0; i < c; ++i) std::memcpy(l + 4 + 8 * i, &entries[i], 8);
  }

  // hnsw.hh:40-251
  void insert(u32 id, const f32* components, u32 drawn_level, u32 shard) {
    u32 new_node_level = drawn_level;  // :48 (drawn by the caller in slot order)
    bool allocated = false;
    u64 new_node_ptr = 0;
    if (cached_ep_ptr == 0) {
      cached_ep_ptr = I.ep_ptr();  // :57
      if (cached_ep_ptr == 0) {    // :60 index not yet initialised
        new_node_level = 0;
        new_node_ptr = allocate_node(new_node_level, shard);                   // :62
        write_node(new_node_ptr, id, components, new_node_level, HEADER_NODE_LOCK);  // :63
        allocated = true;
        I.set_ep_ptr(new_node_ptr);  // :69 CAS succeeds (single writer)
        I.set_header(new_node_ptr, HEADER_ENTRY_NODE);  // :72
        cached_ep_ptr = new_node_ptr;
        return;  // :77
      }
    }
    const u64 entry_point = cached_ep_ptr;  // :88 (single writer: cached pointer is always current)
    I.set_header(entry_point, I.header(entry_point) | HEADER_NEW_LEVEL_LOCK);  // :89-96
    const u32 top_level = I.level(entry_point);
    const bool is_new_level = new_node_level > top_level;  // :101
    if (!is_new_level) {
      I.set_header(entry_point, I.header(entry_point) & ~u64{0xFF00});  // :104 byte 1 := 0
    } else {
      new_node_level = top_level + 1;  // :106
    }
    if (new_node_level > I.max_level) I.max_level = new_node_level;  // :110
    if (!allocated) {
      new_node_ptr = allocate_node(new_node_level, shard);                         // :114
      write_node(new_node_ptr, id, components, new_node_level, HEADER_NODE_LOCK);  // :115
    }
    const f32 ep_distance = I.dist(components, I.comps(entry_point));  // :123
    ++I.build_distcomps;
    MaxHeap& top = st.top_candidates;
    if (new_node_level < top_level) {  // :129
      u64 nn = entry_point;
      const u64 before = st.distcomps;
      search_for_one(I, components, nn, ep_distance, top_level, new_node_level, st);
      I.build_distcomps += st.distcomps - before;
      st.distcomps = before;
      top.push({nn, I.dist(I.comps(nn), components)});  // :138
      ++I.build_distcomps;
    } else {
      top.push({entry_point, ep_distance});  // :142
    }
    if (is_new_level) --new_node_level;  // :146-148
    for (int32_t current_level = static_cast<int32_t>(new_node_level); current_level >= 0; --current_level) {
      const u32 cl = static_cast<u32>(current_level);
      {
        const u64 before = st.distcomps;
        search_level(I, components, efc, cl, st);  // :153
        I.build_distcomps += st.distcomps - before;
        st.distcomps = before;
      }
      select_heuristic(I, top, I.L.m);  // :163
      {                                 // :165-175 write own list in heap-array order
        std::vector<u64> own;
        for (const auto& e : top.heap) own.push_back(e.node);
        write_list(new_node_ptr, cl, own);
      }
      const u32 m_max = cl == 0 ? I.L.m_max_zero : I.L.m_max;  // :177
      for (const auto& [neighbor, neighbor_dist] : top.heap) {  // :180
        const u8* nl = I.list(neighbor, cl);                   // :189-191
        const u32 cnt = Index::list_count(nl);
        if (cnt < m_max) {  // :193-195 append + write count and last entry
          u8* l = I.list_mut(neighbor, cl);
          std::memcpy(l + 4 + 8 * cnt, &new_node_ptr, 8);
          const u32 c1 = cnt + 1;
          std::memcpy(l, &c1, 4);
        } else {  // :197-222 shrink connections
          MaxHeap new_neighbors;
          new_neighbors.push({new_node_ptr, neighbor_dist});  // :202
          for (u32 i = 0; i < cnt; ++i) {                     // :204-209
            const u64 old = Index::list_at(nl, i);
            new_neighbors.push({old, I.dist(I.comps(neighbor), I.comps(old))});
            ++I.build_distcomps;
          }
          select_heuristic(I, new_neighbors, m_max);  // :212
          std::vector<u64> nn;
          for (const auto& e : new_neighbors.heap) nn.push_back(e.node);  // :215-218
          write_list(neighbor, cl, nn);                                      // :221
        }
      }
      while (current_level > 0 && top.size() > 1) top.pop();  // :228-230
    }
    I.set_header(new_node_ptr, is_new_level ? HEADER_ENTRY_NODE : 0);  // :234
    if (is_new_level) {
      I.set_header(entry_point, I.header(entry_point) & ~u64{0xFF0000});  // :238 byte 2 := 0
      I.set_header(entry_point, I.header(entry_point) & ~u64{0xFF00});    // :239 byte 1 := 0
      I.set_ep_ptr(new_node_ptr);                                          // :244
      cached_ep_ptr = new_node_ptr;
    }
    top.clear();  // :250
  }
};

}  // namespace oracle

// ============================================================================================================
//  C ABI for the Python test harness (ctypes)
// ============================================================================================================
using namespace oracle;

extern "C" {

// Level draw exactly as hnsw.hh:30,34-35,48: floor(-ln(U(0,1)) * 1/ln(M)) with std::mt19937(seed) and
// std::uniform_real_distribution<double>; the memory node per insert from a seeded std::mt19937 and
// std::uniform_int_distribution<u32>(0, n-1) (compute_thread.hh:39,57 draws it from a random_device seed).
void oracle_draw_levels(uint32_t n, uint32_t M, uint32_t seed, uint32_t n_shards, uint32_t* levels,
                        uint32_t* shards) {
  std::mt19937 prng(seed);
  std::uniform_real_distribution<> uniform(0., 1.);
  const f64 nf = 1. / std::log(static_cast<f64>(M));
  std::mt19937 shard_rng(seed ^ 0x9E3779B9u);
  std::uniform_int_distribution<u32> sd(0, n_shards - 1);
  for (u32 i = 0; i < n; ++i) {
    levels[i] = static_cast<u32>(std::floor(-std::log(uniform(prng)) * nf));
    shards[i] = sd(shard_rng);
  }
}

// Builds the index by inserting base[0..n) in slot order.  Returns an opaque handle.
void* oracle_build(const float* base, uint32_t n, uint32_t dim, uint32_t M, uint32_t efc, int metric,
                   uint32_t n_shards, uint32_t seed) {
  auto* I = new Index();
  I->L.init(dim, M);
  I->metric = metric;
  std::vector<u32> levels(n), shard_of(n);
  oracle_draw_levels(n, M, seed, n_shards, levels.data(), shard_of.data());
  // size each shard buffer for the drawn levels (effective level <= drawn level + 0; new levels cap at +1)
  std::vector<u64> cap(n_shards, 16);
  for (u32 i = 0; i < n; ++i) cap[shard_of[i]] += I->L.alloc_size(levels[i] + 1);
  I->shards.resize(n_shards);
  for (u32 s = 0; s < n_shards; ++s) I->shards[s].assign(cap[s], 0);
  Builder b(*I, efc);
  b.free_ptr.assign(n_shards, 16);  // memory_node.hh:61
  for (u32 s = 0; s < n_shards; ++s) std::memcpy(I->shards[s].data(), &b.free_ptr[s], 8);
  for (u32 i = 0; i < n; ++i) b.insert(i, base + static_cast<size_t>(i) * dim, levels[i], shard_of[i]);
  for (u32 s = 0; s < n_shards; ++s) I->shards[s].resize(b.free_ptr[s]);  // dump = [0, free_ptr)
  return I;
}

uint64_t oracle_dump_size(void* h, uint32_t shard) { return static_cast<Index*>(h)->shards[shard].size(); }
const uint8_t* oracle_dump_data(void* h, uint32_t shard) { return static_cast<Index*>(h)->shards[shard].data(); }
uint64_t oracle_build_distcomps(void* h) { return static_cast<Index*>(h)->build_distcomps; }
uint32_t oracle_max_level(void* h) { return static_cast<Index*>(h)->max_level; }

// Opens dumps (memory_node.hh:157-183 loads them verbatim).  dim / M / metric are not stored in the file.
void* oracle_open(const uint8_t* const* bufs, const uint64_t* sizes, uint32_t n_shards, uint32_t dim,
                  uint32_t M, int metric) {
  auto* I = new Index();
  I->L.init(dim, M);
  I->metric = metric;
  I->shards.resize(n_shards);
  for (u32 s = 0; s < n_shards; ++s) I->shards[s].assign(bufs[s], bufs[s] + sizes[s]);
  return I;
}

void oracle_free(void* h) { delete static_cast<Index*>(h); }

// knn over a batch; queries are processed by n_threads worker threads (one query per thread at a time,
// like `--threads T --coroutines 1`), each with its own SearchState.  stats: nq × 8 u32 (QS_* layout).
// cpus (nullable): worker t is pinned to CPU cpus[t] (the reference pins its compute threads to cores,
// compute_node.cc:362-380, core_assignment.hh:22-44); timing only, results do not depend on it.
int oracle_knn_pinned(void* h, const float* queries, uint32_t nq, uint32_t k, uint32_t ef, uint32_t* out_ids,
                      float* out_dists, uint32_t* stats, uint32_t n_threads, const int32_t* cpus) {
  const Index& I = *static_cast<Index*>(h);
  if (ef < k) return 1;  // hnsw.hh:36 lib_assert(ef_search >= k)
  if (I.ep_ptr() == 0) return 2;
  std::atomic<u32> next{0};
  auto pin = [&](u32 t) {
    if (!cpus) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpus[t], &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  };
  auto worker = [&]() {
    SearchState st;
    for (;;) {
      const u32 qi = next.fetch_add(1);
      if (qi >= nq) break;
      knn(I, queries + static_cast<size_t>(qi) * I.L.dim, k, ef, st, out_ids + static_cast<size_t>(qi) * k,
          out_dists ? out_dists + static_cast<size_t>(qi) * k : nullptr);
      if (stats) std::memcpy(stats + static_cast<size_t>(qi) * QS_WORDS, st.qs, sizeof(st.qs));
    }
  };
  if (n_threads <= 1 && !cpus) {
    worker();
  } else {
    std::vector<std::thread> ts;
    for (u32 t = 0; t < std::max<u32>(1, n_threads); ++t) ts.emplace_back([&, t]() { pin(t); worker(); });
    for (auto& t : ts) t.join();
  }
  return 0;
}

int oracle_knn(void* h, const float* queries, uint32_t nq, uint32_t k, uint32_t ef, uint32_t* out_ids,
               float* out_dists, uint32_t* stats, uint32_t n_threads) {
  return oracle_knn_pinned(h, queries, nq, k, ef, out_ids, out_dists, stats, n_threads, nullptr);
}

// knn with the record reads of every query (single thread): reads[offsets[i] .. offsets[i+1]) are query i's node
// reads in order, each (uid << 1) | always, where always = 1 for the entry point and upper-level nodes (admitted
// without the coin, hnsw.hh:263, 368) and 0 for level-0 neighbours (hnsw.hh:447-448); nodes[] the memory node of
// each read.  Returns 3 when cap is too small.  The reads are what a compute-node cache sees (cache_lookup).
int oracle_knn_trace(void* h, const float* queries, uint32_t nq, uint32_t k, uint32_t ef, uint32_t* out_ids,
                     float* out_dists, uint32_t* stats, uint32_t* reads, uint16_t* nodes, uint64_t cap,
                     uint64_t* offsets) {
  const Index& I = *static_cast<Index*>(h);
  if (ef < k) return 1;
  if (I.ep_ptr() == 0) return 2;
  SearchState st;
  std::vector<std::pair<u64, bool>> rd;
  st.reads = &rd;
  uint64_t n = 0;
  offsets[0] = 0;
  for (u32 qi = 0; qi < nq; ++qi) {
    rd.clear();
    knn(I, queries + static_cast<size_t>(qi) * I.L.dim, k, ef, st, out_ids + static_cast<size_t>(qi) * k,
        out_dists ? out_dists + static_cast<size_t>(qi) * k : nullptr);
    if (stats) std::memcpy(stats + static_cast<size_t>(qi) * QS_WORDS, st.qs, sizeof(st.qs));
    if (n + rd.size() > cap) return 3;
    for (const auto& [r, always] : rd) {
      reads[n] = (I.uid(r) << 1) | (always ? 1u : 0u);
      nodes[n] = static_cast<uint16_t>(rp_node(r));
      ++n;
    }
    offsets[qi + 1] = n;
  }
  return 0;
}

// Distances of explicit (query, node-uid) pairs, for distance-kernel parity.  node_uids index the dense
// record order of shard 0..n (the order records appear in the dumps).
float oracle_distance(int metric, const float* a, const float* b, uint32_t dim) {
  return distance(metric, a, b, dim);
}

// The as-written form (its rounding is whatever this build's flags make of it; see l2_as_written), called out of
// line, one pair per call.
__attribute__((noinline)) float oracle_distance_as_written(int metric, const float* a, const float* b, uint32_t dim) {
#ifdef ORACLE_AVX2
  return metric == 1 ? ip_as_written(a, b, dim) : l2_as_written(a, b, dim);
#else
  return distance(metric, a, b, dim);
#endif
}

// The same as-written form in another context: distance() inlined into a loop over n pairs, as the reference's
// search loops call Distance::dist (hnsw.hh:376, 458).  Under -ffast-math the two contexts may round differently.
void oracle_distances_in_loop(int metric, const float* a, const float* b, uint32_t n, uint32_t dim, float* out) {
  for (uint32_t i = 0; i < n; ++i)
    out[i] = distance(metric, a + static_cast<size_t>(i) * dim, b + static_cast<size_t>(i) * dim, dim);
}

// ---- libstdc++ pinning hooks: run the SAME std:: calls on caller data so the tests can compare the GPU's
// re-implementation of push_heap / pop_heap / make_heap against libstdc++ on adversarial (tied) inputs.
// ops: 0 = push(value), 1 = pop, 2 = push_k(value, k) ; is_max selects MaxHeapCompare / MinHeapCompare.
int oracle_selftest_heap(int is_max, const int32_t* ops, const float* vals, const uint32_t* ids, uint32_t n_ops,
                         uint32_t k, float* out_d, uint32_t* out_id, uint32_t* out_n) {
  auto run = [&](auto& H) {
    for (u32 i = 0; i < n_ops; ++i) {
      const Entry e{ids[i], vals[i]};
      if (ops[i] == 0) H.push(e);
      else if (ops[i] == 1) { if (!H.empty()) H.pop(); }
      else H.push_k(e, k);
    }
    *out_n = static_cast<u32>(H.size());
    for (size_t i = 0; i < H.size(); ++i) { out_d[i] = H.heap[i].distance; out_id[i] = static_cast<u32>(H.heap[i].node); }
  };
  if (is_max) { MaxHeap H; run(H); } else { MinHeap H; run(H); }
  return 0;
}

}  // extern "C"
