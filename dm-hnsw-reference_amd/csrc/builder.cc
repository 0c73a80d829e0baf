// Build path: parallel CPU restatement of HNSW::insert (src/hnsw/hnsw.hh:40-251) that
// writes the memory nodes' buffers `[free_ptr | ep_ptr | records...]` (src/memory_node.hh:15-27) directly,
// i.e. the same bytes `--store-index` dumps (memory_node.hh:185-201).
//
// Concurrency follows the reference protocol, with the RDMA verbs replaced by host atomics on the same words:
//   * FAA on each memory node's free_ptr to allocate a record          (rdma_atomics.hh:88-130)
//   * CAS on the entry-point pointer to initialise the index            (rdma_atomics.hh:132-154)
//   * CAS on the record header's lock / new-level-lock bits             (rdma_atomics.hh:13-86)
//   * single-byte stores to release them                                (rdma_writes.hh:14-72)
// With threads == 1 the insert order is the slot order and the output is byte-identical to the oracle's
// single-threaded build (tests/test_builder.py).  Level draws are made up front in slot order from the same
// std::mt19937(seed) / uniform_real_distribution<double> stream (hnsw.hh:34-35,48), and the memory node of
// each record from a seeded std::mt19937 (the reference seeds it from std::random_device,
// compute_thread.hh:88), so both are independent of thread interleaving.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <random>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>


#include "../../include/shine_gpu.h"
#include "graph.h"
#include "hostdist.h"

namespace shine {
namespace {

constexpr u64 kLock = 0b01;                    // node.hh:28
constexpr u64 kNewLevelLock = 0b100000000;     // node.hh:29
constexpr u64 kEntryNode = 0b10000000000000000;// node.hh:30

struct Entry {
  u64 node;
  f32 distance;
};
struct MaxCmp {
  bool operator()(const Entry& l, const Entry& r) const { return l.distance < r.distance; }
};
struct MinCmp {
  bool operator()(const Entry& l, const Entry& r) const { return l.distance > r.distance; }
};

// Exact visited set keyed by RemotePtr (types.hh:14-15): open addressing, generation-tagged so clear() is O(1).
class VisitedSet {
 public:
  bool insert(u64 key) {  // true if newly inserted
    if ((size_ + 1) * 2 > keys_.size()) grow();
    const size_t mask = keys_.size() - 1;
    size_t i = hash(key) & mask;
    while (gen_[i] == cur_) {
      if (keys_[i] == key) return false;
      i = (i + 1) & mask;
    }
    gen_[i] = cur_;
    keys_[i] = key;
    ++size_;
    return true;
  }
  void clear() {
    ++cur_;
    size_ = 0;
    if (cur_ == 0) {
      std::fill(gen_.begin(), gen_.end(), 0);
      cur_ = 1;
    }
  }

 private:
  static size_t hash(u64 h) {  // remote_pointer.hh:31-51 (murmur64 finaliser)
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return static_cast<size_t>(h);
  }
  void grow() {
    std::vector<u64> ok;
    ok.reserve(size_);
    for (size_t i = 0; i < keys_.size(); ++i)
      if (gen_[i] == cur_) ok.push_back(keys_[i]);
    const size_t n = std::max<size_t>(1024, keys_.size() * 2);
    keys_.assign(n, 0);
    gen_.assign(n, 0);
    cur_ = 1;
    size_ = 0;
    for (u64 k : ok) insert(k);
  }
  std::vector<u64> keys_;
  std::vector<uint32_t> gen_;
  uint32_t cur_ = 1;
  size_t size_ = 0;
};

struct ThreadState {
  VisitedSet visited;
  std::vector<Entry> top, next;  // MaxHeap top_candidates / MinHeap next_candidates (coroutine.hh:60-62)
  u64 cached_ep_ptr = 0;
  u64 distcomps = 0;
};

class ParallelBuilder {
 public:
  ParallelBuilder(const f32* base, u64 n, u32 dim, u32 M, u32 efc, int metric, u32 n_shards, u32 seed)
      : base_(base), n_(n), efc_(efc), metric_(metric), n_shards_(n_shards) {
    L_.dim = dim;
    L_.M = M;
    levels_.resize(n);
    shard_of_.resize(n);
    std::mt19937 prng(seed);                     // hnsw.hh:34 (seed = --seed + client_id)
    std::uniform_real_distribution<> uniform(0., 1.);
    const double nf = 1. / std::log(static_cast<double>(M));  // hnsw.hh:30
    std::mt19937 shard_rng(seed ^ 0x9E3779B9u);
    std::uniform_int_distribution<u32> sd(0, n_shards - 1);
    for (u64 i = 0; i < n; ++i) {
      levels_[i] = static_cast<u32>(std::floor(-std::log(uniform(prng)) * nf));  // hnsw.hh:48
      shard_of_[i] = sd(shard_rng);
    }
    std::vector<u64> cap(n_shards, 16);
    for (u64 i = 0; i < n; ++i) cap[shard_of_[i]] += L_.alloc_size(levels_[i] + 1);
    shards_.resize(n_shards);
    free_ptr_ = std::make_unique<std::atomic<u64>[]>(n_shards);
    for (u32 s = 0; s < n_shards; ++s) {
      shards_[s].assign(cap[s], 0);
      free_ptr_[s].store(16);  // memory_node.hh:61
    }
  }

  void run(u32 threads) {
    std::atomic<u64> next_idx{0};  // compute_node.hh next_insert_idx_ (scheduler.hh:56 fetch_add)
    auto worker = [&]() {
      ThreadState st;
      for (;;) {
        const u64 slot = next_idx.fetch_add(1);
        if (slot >= n_) break;
        insert(static_cast<u32>(slot), base_ + slot * L_.dim, levels_[slot], shard_of_[slot], st);
      }
      distcomps_.fetch_add(st.distcomps);
    };
    if (threads <= 1) {
      worker();
    } else {
      std::vector<std::thread> ts;
      for (u32 t = 0; t < threads; ++t) ts.emplace_back(worker);
      for (auto& t : ts) t.join();
    }
    for (u32 s = 0; s < n_shards_; ++s) {
      const u64 fp = free_ptr_[s].load();
      std::memcpy(shards_[s].data(), &fp, 8);
      shards_[s].resize(fp);
    }
  }

  std::vector<std::vector<u8>> shards_;
  std::atomic<u64> distcomps_{0};

 private:
  // ---- memory-node words --------------------------------------------------------------------------------
  u8* at(u64 r) { return shards_[r >> 48].data() + ((r << 16) >> 16); }
  u64* hdr(u64 r) { return reinterpret_cast<u64*>(at(r)); }  // records are 8-byte aligned (rdma_atomics.hh:92)
  u64 load_hdr(u64 r) { return __atomic_load_n(hdr(r), __ATOMIC_ACQUIRE); }
  u32 level(u64 r) { u32 v; std::memcpy(&v, at(r) + 12, 4); return v; }
  u32 uid(u64 r) { u32 v; std::memcpy(&v, at(r) + 8, 4); return v; }
  const f32* comps(u64 r) { return reinterpret_cast<const f32*>(at(r) + 16); }
  u8* list(u64 r, u32 l) { return shards_[r >> 48].data() + L_.list_offset((r << 16) >> 16, l); }
  u64* ep_word() { return reinterpret_cast<u64*>(shards_[0].data() + 8); }
  static u32 list_count(const u8* l) { u32 c; std::memcpy(&c, l, 4); return c; }
  static u64 list_at(const u8* l, u32 i) { u64 v; std::memcpy(&v, l + 4 + 8ull * i, 8); return v; }

  f32 dist(const f32* a, const f32* b) { return metric_ == 1 ? host_ip(a, b, L_.dim) : host_l2(a, b, L_.dim); }

  // rdma_atomics.hh:49-61 spinlock_node: CAS(header & ~lock → | lock) until it succeeds
  void lock_node(u64 r) {
    u64 expected = load_hdr(r) & ~kLock;
    for (;;) {
      u64 cmp = expected & ~kLock;
      if (__atomic_compare_exchange_n(hdr(r), &cmp, cmp | kLock, false, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) return;
      expected = cmp;  // node->header() = original_header
      std::this_thread::yield();
    }
  }
  // rdma_writes.hh:14-32 unlock_node: write byte 0 := 0
  void unlock_node(u64 r) { __atomic_store_n(reinterpret_cast<u8*>(hdr(r)), u8{0}, __ATOMIC_RELEASE); }
  void unlock_new_level(u64 r) { __atomic_store_n(reinterpret_cast<u8*>(hdr(r)) + 1, u8{0}, __ATOMIC_RELEASE); }
  void clear_entry_bit(u64 r) { __atomic_store_n(reinterpret_cast<u8*>(hdr(r)) + 2, u8{0}, __ATOMIC_RELEASE); }

  u64 allocate_node(u32 lvl, u32 shard) {  // rdma_atomics.hh:88-130
    const u64 sz = L_.alloc_size(lvl);
    const u64 off = free_ptr_[shard].fetch_add(sz);
    return (static_cast<u64>(shard) << 48) | off;
  }
  void write_node(u64 r, u32 id, const f32* c, u32 lvl, u64 header) {  // rdma_writes.hh:75-124
    u8* p = at(r);
    std::memcpy(p + 8, &id, 4);
    std::memcpy(p + 12, &lvl, 4);
    std::memcpy(p + 16, c, 4ull * L_.dim);
    __atomic_store_n(reinterpret_cast<u64*>(p), header, __ATOMIC_RELEASE);
  }
  void write_list(u64 r, u32 l, const std::vector<Entry>& es) {  // rdma_writes.hh:151-171
    u8* p = list(r, l);
    const u32 c = static_cast<u32>(es.size());
    for (u32 i = 0; i < c; ++i) std::memcpy(p + 4 + 8ull * i, &es[i].node, 8);
    std::memcpy(p, &c, 4);
  }

  // hnsw.hh:331-393 with_lock
  void search_for_one(const f32* q, u64& nn, f32 closest, u32 begin, u32 target, ThreadState& st) {
    bool changed;
    for (u32 lv = begin; lv > target; lv--) {
      do {
        changed = false;
        const u64 locked = nn;
        lock_node(locked);
        const u8* nl = list(nn, lv);
        u64 best = 0;
        const u32 cnt = list_count(nl);
        for (u32 i = 0; i < cnt; ++i) {
          const u64 c = list_at(nl, i);
          const f32 d = dist(q, comps(c));
          ++st.distcomps;
          if (d < closest) {
            closest = d;
            best = c;
            changed = true;
          }
        }
        nn = changed ? best : nn;
        unlock_node(locked);
      } while (changed);
    }
  }

  // hnsw.hh:406-476 with_lock
  void search_level(const f32* q, u32 ef, u32 lv, ThreadState& st) {
    auto& top = st.top;
    auto& next = st.next;
    for (const auto& e : top) {
      next.push_back(e);
      std::push_heap(next.begin(), next.end(), MinCmp());
      st.visited.insert(e.node);
    }
    while (!next.empty()) {
      const Entry c = next.front();
      std::pop_heap(next.begin(), next.end(), MinCmp());
      next.pop_back();
      if (c.distance > top.front().distance) break;
      lock_node(c.node);
      const u8* nl = list(c.node, lv);
      const u32 cnt = list_count(nl);
      for (u32 i = 0; i < cnt; ++i) {
        const u64 nb = list_at(nl, i);
        if (!st.visited.insert(nb)) continue;
        const f32 farthest = top.front().distance;
        const f32 nd = dist(q, comps(nb));
        ++st.distcomps;
        if (nd < farthest || top.size() < ef) {
          next.push_back({nb, nd});
          std::push_heap(next.begin(), next.end(), MinCmp());
          if (top.size() < ef) {  // heap.hh:34-41
            top.push_back({nb, nd});
            std::push_heap(top.begin(), top.end(), MaxCmp());
          } else if (nd < top.front().distance) {
            std::pop_heap(top.begin(), top.end(), MaxCmp());
            top.pop_back();
            top.push_back({nb, nd});
            std::push_heap(top.begin(), top.end(), MaxCmp());
          }
        }
      }
      unlock_node(c.node);
    }
    next.clear();
    st.visited.clear();
  }

  // hnsw.hh:482-522
  void select_heuristic(std::vector<Entry>& top, u32 m, ThreadState& st) {
    if (top.size() < m) return;
    std::sort(top.begin(), top.end(), [&](const Entry& l, const Entry& r) {
      return l.distance == r.distance ? uid(l.node) < uid(r.node) : l.distance < r.distance;
    });
    const size_t initial = top.size();
    size_t selected = 1, consumed = 1;
    while (selected < m && consumed < initial) {
      bool is_selected = true;
      const Entry c = top[consumed];
      for (size_t i = 0; i < selected; ++i) {
        const f32 d = dist(comps(top[i].node), comps(c.node));
        ++st.distcomps;
        if (d < c.distance) {
          is_selected = false;
          break;
        }
      }
      if (is_selected) {
        std::swap(top[selected], top[consumed]);
        ++selected;
      }
      ++consumed;
    }
    top.resize(selected);
    std::make_heap(top.begin(), top.end(), MaxCmp());
  }

  // hnsw.hh:40-251
  void insert(u32 id, const f32* components, u32 drawn_level, u32 shard, ThreadState& st) {
    u32 new_level = drawn_level;
    bool allocated = false;
    u64 new_ptr = 0;
    u64& cached = st.cached_ep_ptr;
    if (cached == 0) {
      cached = __atomic_load_n(ep_word(), __ATOMIC_ACQUIRE);  // :57
      if (cached == 0) {
        new_level = 0;
        new_ptr = allocate_node(new_level, shard);
        write_node(new_ptr, id, components, new_level, kLock);
        allocated = true;
        u64 expected = 0;
        if (__atomic_compare_exchange_n(ep_word(), &expected, new_ptr, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
          __atomic_store_n(hdr(new_ptr), kEntryNode, __ATOMIC_RELEASE);  // :72
          cached = new_ptr;
          return;
        }
        cached = expected;  // lost the race (:80)
      }
    }
    // lock_and_update_entry_point (rdma_atomics.hh:67-86)
    u64 ep;
    for (;;) {
      ep = cached;
      u64 h = load_hdr(ep);
      while (!(h & kEntryNode)) {
        cached = __atomic_load_n(ep_word(), __ATOMIC_ACQUIRE);
        ep = cached;
        h = load_hdr(ep);
      }
      u64 cmp = h & ~kNewLevelLock;
      if (__atomic_compare_exchange_n(hdr(ep), &cmp, cmp | kNewLevelLock, false, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED))
        break;
      std::this_thread::yield();
    }
    const u32 top_level = level(ep);
    const bool is_new_level = new_level > top_level;
    if (!is_new_level) unlock_new_level(ep);
    else new_level = top_level + 1;
    if (!allocated) {
      new_ptr = allocate_node(new_level, shard);
      write_node(new_ptr, id, components, new_level, kLock);
    }
    const f32 ep_distance = dist(components, comps(ep));
    ++st.distcomps;
    auto& top = st.top;
    if (new_level < top_level) {
      u64 nn = ep;
      search_for_one(components, nn, ep_distance, top_level, new_level, st);
      top.push_back({nn, dist(comps(nn), components)});
      std::push_heap(top.begin(), top.end(), MaxCmp());
      ++st.distcomps;
    } else {
      top.push_back({ep, ep_distance});
      std::push_heap(top.begin(), top.end(), MaxCmp());
    }
    if (is_new_level) --new_level;
    std::vector<Entry> nbrs;
    for (int32_t cl_i = static_cast<int32_t>(new_level); cl_i >= 0; --cl_i) {
      const u32 cl = static_cast<u32>(cl_i);
      search_level(components, efc_, cl, st);
      select_heuristic(top, L_.M, st);
      write_list(new_ptr, cl, top);
      const u32 m_max = cl == 0 ? 2 * L_.M : L_.M;
      for (const auto& [neighbor, neighbor_dist] : top) {
        lock_node(neighbor);
        u8* nl = list(neighbor, cl);
        const u32 cnt = list_count(nl);
        if (cnt < m_max) {
          std::memcpy(nl + 4 + 8ull * cnt, &new_ptr, 8);
          const u32 c1 = cnt + 1;
          std::memcpy(nl, &c1, 4);
        } else {
          nbrs.clear();
          nbrs.push_back({new_ptr, neighbor_dist});
          std::push_heap(nbrs.begin(), nbrs.end(), MaxCmp());
          for (u32 i = 0; i < cnt; ++i) {
            const u64 old = list_at(nl, i);
            nbrs.push_back({old, dist(comps(neighbor), comps(old))});
            std::push_heap(nbrs.begin(), nbrs.end(), MaxCmp());
            ++st.distcomps;
          }
          select_heuristic(nbrs, m_max, st);
          write_list(neighbor, cl, nbrs);
        }
        unlock_node(neighbor);
      }
      while (cl_i > 0 && top.size() > 1) {
        std::pop_heap(top.begin(), top.end(), MaxCmp());
        top.pop_back();
      }
    }
    __atomic_store_n(hdr(new_ptr), is_new_level ? kEntryNode : u64{0}, __ATOMIC_RELEASE);  // :234
    if (is_new_level) {
      clear_entry_bit(ep);      // :238
      unlock_new_level(ep);     // :239
      __atomic_store_n(ep_word(), new_ptr, __ATOMIC_RELEASE);  // :244
      cached = new_ptr;
    }
    top.clear();
  }

  const f32* base_;
  u64 n_;
  u32 efc_;
  int metric_;
  u32 n_shards_;
  RecordLayout L_;
  std::vector<u32> levels_, shard_of_;
  std::unique_ptr<std::atomic<u64>[]> free_ptr_;
};

}  // namespace
}  // namespace shine

struct shine_build {
  std::vector<std::vector<uint8_t>> shards;
  uint64_t distcomps = 0;
};

extern "C" {

int shine_build(const float* base, uint64_t n, uint32_t dim, uint32_t M, uint32_t ef_construction, int metric,
                uint32_t n_shards, uint32_t seed, uint32_t threads, shine_build_t* out) {
  using namespace shine;
  if (!out || !base) return set_error(SHINE_ERR_ARG, "NULL argument");
  if (n == 0 || n >= 0xFFFFFFFFull) return set_error(SHINE_ERR_ARG, "n must be in [1, 2^32-1)");
  if (dim == 0 || M < 2 || M > 32 || ef_construction == 0 || n_shards == 0 || n_shards > 65535)
    return set_error(SHINE_ERR_ARG, "invalid build parameters (dim>0, 2<=M<=32, efC>0, 1<=shards<=65535)");
  if (metric != SHINE_METRIC_L2 && metric != SHINE_METRIC_IP) return set_error(SHINE_ERR_ARG, "metric must be 0 or 1");
  if (threads == 0) threads = std::max(1u, std::thread::hardware_concurrency());
  try {
    ParallelBuilder b(base, n, dim, M, ef_construction, metric, n_shards, seed);
    b.run(threads);
    auto* r = new struct shine_build();
    r->shards = std::move(b.shards_);
    r->distcomps = b.distcomps_.load();
    *out = r;
  } catch (const std::bad_alloc&) {
    return set_error(SHINE_ERR_NOMEM, "out of host memory while building");
  }
  return SHINE_OK;
}

uint64_t shine_build_dump_size(shine_build_t b, uint32_t s) { return b && s < b->shards.size() ? b->shards[s].size() : 0; }
const uint8_t* shine_build_dump_data(shine_build_t b, uint32_t s) {
  return b && s < b->shards.size() ? b->shards[s].data() : nullptr;
}
uint64_t shine_build_distcomps(shine_build_t b) { return b ? b->distcomps : 0; }

// compute_node.cc:426-430: <dir>/dump/index_m{M}_efc{efC}_node{i}_of{N}.dat
int shine_build_write(shine_build_t b, const char* dir, uint32_t M, uint32_t efc) {
  using namespace shine;
  if (!b || !dir) return set_error(SHINE_ERR_ARG, "NULL argument");
  const std::string d = std::string(dir) + "/dump";
  mkdir(dir, 0755);
  mkdir(d.c_str(), 0755);
  const size_t N = b->shards.size();
  for (size_t i = 0; i < N; ++i) {
    const std::string p = d + "/index_m" + std::to_string(M) + "_efc" + std::to_string(efc) + "_node" +
                          std::to_string(i + 1) + "_of" + std::to_string(N) + ".dat";
    std::ofstream f(p, std::ios::binary);
    if (!f.write(reinterpret_cast<const char*>(b->shards[i].data()), static_cast<std::streamsize>(b->shards[i].size())))
      return set_error(SHINE_ERR_IO, "cannot write " + p);
  }
  return SHINE_OK;
}

int shine_build_free(shine_build_t b) {
  delete b;
  return SHINE_OK;
}

}  // extern "C"
