// Internal to libshine_gpu.so: the index handle's state (capi.cc) shared with the GPU batch builder (gpu_build.cc).
// Nothing here crosses the C ABI (include/shine_gpu.h).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/shine_gpu.h"
#include "cache.h"
#include "graph.h"
#include "kernels.h"
#include "placement.h"
#include "views.h"

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t _e = (expr);                                                                        \
    if (_e != hipSuccess)                                                                          \
      return ::shine::set_error(_e == hipErrorOutOfMemory ? SHINE_ERR_NOMEM : SHINE_ERR_HIP,       \
                                std::string(#expr) + ": " + hipGetErrorString(_e));                \
  } while (0)

struct shine_index;
struct shine_request;

namespace shine {

constexpr uint32_t kLogCap = 32768;          // visited ids remembered per slot for O(visited) clearing
constexpr uint64_t kBitmapBudget = 1ull << 30;  // HBM for the fallback passes' visited bitmaps, per stream
constexpr uint32_t kGlobalNextCap = 131072;  // next_candidates capacity of the global-heap pass (1 MiB per slot)
constexpr uint32_t kGlobalSlots = 64;        // persistent slots of the global-heap pass (it sees few queries)

// Pinned host staging (shine_knn_batch): asynchronous copies, no pageable bounce.
template <class T>
struct HostBuf {
  T* p = nullptr;
  size_t n = 0;
  int grow(size_t want, unsigned flags = hipHostMallocDefault) {
    if (want <= n) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(want, 1) * sizeof(T), flags);
    if (e != hipSuccess) return set_error(SHINE_ERR_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    std::memset(p, 0, std::max<size_t>(want, 1) * sizeof(T));
    n = want;
    return 0;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  int grow(size_t want) {
    if (want <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(want, 1) * sizeof(T));
    if (e != hipSuccess)
      return set_error(e == hipErrorOutOfMemory ? SHINE_ERR_NOMEM : SHINE_ERR_HIP,
                       std::string("hipMalloc: ") + hipGetErrorString(e));
    n = want;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// A reserved virtual range and the pieces mapped into it (one GPU's view of a sharded array, see ShardedArray).
struct StripedRange {
  char* va = nullptr;
  size_t bytes = 0;  // reserved
  std::vector<std::pair<size_t, size_t>> maps;  // (offset, size) of each mapped piece
  std::vector<hipMemGenericAllocationHandle_t> handles;
  void release() {
    for (auto& m : maps) (void)hipMemUnmap(va + m.first, m.second);
    for (auto& hd : handles) (void)hipMemRelease(hd);
    if (va) (void)hipMemAddressFree(va, bytes);
    maps.clear();
    handles.clear();
    va = nullptr;
    bytes = 0;
  }
};

// A sharded level-0 array (vectors or lists; SHINE_PLACE_SHARDED).  Slot o owns the rows o*U .. o*U+U-1 of the id
// space, ordered hottest first, in two physical allocations on its GPU: hot[o] (the first `cached` bytes) and
// cold[o] (the rest).  Every slot has its own view of the whole id space: its own stripe, local copies of every
// other slot's hot prefix (copy[o]: the cache of remote records, ≙ cache::Cache, cache.hh:102-311) and the other
// slots' cold rows mapped to their owners' HBM (xGMI peer reads).  Mappings start at offset 0 of a handle.
struct ShardedArray {
  uint64_t stride = 0;  // U * row bytes, a multiple of the VM granularity
  size_t cached = 0;    // bytes of each stripe that other slots keep local copies of (0 = no cache)
  std::vector<hipMemGenericAllocationHandle_t> hot, cold, copy;  // [slot]; unused entries stay 0
  std::vector<StripedRange> view;                                // [slot]
  void release() {
    for (auto& v : view) v.release();
    view.clear();
    for (auto* hs : {&hot, &cold, &copy})
      for (auto& hd : *hs)
        if (hd) (void)hipMemRelease(hd);
    hot.clear();
    cold.clear();
    copy.clear();
  }
};

// Device scratch of one search call (work-queue heads, overflow lists, visited bitmaps, per-query counters).  Each
// stream a caller enqueues on gets its own, so batches on different streams run concurrently on one GPU.
struct Scratch {
  DevBuf<uint32_t> visited, vlog, counter, ovf, qs;
  DevBuf<uint32_t> spill_flags;  // fast kernel: which of the `visited` bitmaps a spilled query holds (all zero between calls)
  DevBuf<unsigned long long> heaps;  // global-heap pass
  // host memory the last pass of every call writes: [0..2] the queries each pass handed on, [3] = 1 once written,
  // [4] the most nodes a query of that call marked visited (sizes the next call's light pass and visited tables;
  // may be stale while a call is in flight)
  HostBuf<uint32_t> seen;
  uint32_t* seen_dev = nullptr;  // its device address
  bool counters_zero = false;    // the last call's last pass zeroed the counter words (finish_call)
  uint32_t slots = 0;
  uint64_t stride = 0;           // words per slot of `visited` (capi.cc slot_words)
  uint32_t last_table = 0;       // visited-table entries of the last call's main pass, and whether they were learned
  bool last_learned = false;
  uint32_t table_floor = 0;      // a learned table that overflowed is never learned again below twice its size
  uint32_t last_ef = 0;          // ef of the last call: what it visited says nothing about another ef
  uint32_t last_nq = 0;          // queries of the last call (seen[5] / last_nq: the mean a query marked visited)
  bool last_fast = false;        // the last call's main pass was the fast kernel
  bool last_tight = false;       // the last call's exact pass reserved the tight next_candidates room (capi.cc pick_shape)
  uint32_t tight_off_ef = 0;     // ... and handed on more than 1/12 of its queries for it: not again at this ef
  void release() {
    for (auto* b : {&visited, &vlog, &counter, &ovf, &qs, &spill_flags}) b->release();
    heaps.release();
    seen.release();
    seen_dev = nullptr;
    counters_zero = false;
    slots = 0;
    stride = 0;
  }
};

// Pinned staging of one host-API call on one GPU slot, mapped into the GPU's address space (the kernels read the
// queries and write ids, distances and counters there over PCIe), with the device addresses, per-chunk hand-on counts
// and the chunks' completion events.  A slot keeps a pool: a synchronous call takes a set and gives it back before it
// returns, an asynchronous call (shine_knn_batch_async) holds its own until shine_wait, so calls in flight never share.
struct HostStage {
  HostBuf<float> hq, hd;
  HostBuf<uint32_t> hids, hqs, hcnt;  // hcnt: per chunk, queries its passes handed on and a written flag
  float *dq = nullptr, *dd = nullptr;
  uint32_t *dids = nullptr, *dqs = nullptr, *hcnt_dev = nullptr;
  std::vector<hipEvent_t> hchunk;     // chunk c's results are in the staging once hchunk[c] fired
  hipEvent_t ev0 = nullptr;           // before the call's first launch (kernel_ms runs to the last chunk's event)
  void release() {
    for (auto* b : {&hq, &hd}) b->release();
    for (auto* b : {&hids, &hqs, &hcnt}) b->release();
    for (hipEvent_t e : hchunk) (void)hipEventDestroy(e);
    hchunk.clear();
    if (ev0) (void)hipEventDestroy(ev0);
    ev0 = nullptr;
  }
};

struct Replica {
  int device = 0;
  uint32_t slot = 0;
  uint32_t cus = 256;                 // compute units of the device (hipDeviceProp_t, queried at open)
  uint32_t lds_per_cu = 160 * 1024;   // LDS bytes per CU
  uint32_t pad_node = 0;  // a node of this slot's own stripe (sharded) for the unconditional loads of empty slots
  // the worst query's visits of the latest finished call on a stream, as seen at the slot's last 32 enqueues at
  // `vmax_ef` on any of its streams: the learned tables size for the recent batches, not one stream's last
  uint32_t vmax_recent[32] = {};
  uint32_t nmax_recent[32] = {};  // ... and its largest next_candidates (exact passes), at the same enqueues
  uint32_t vmax_pos = 0, vmax_ef = 0;
  uint32_t recent_vmax() const {
    uint32_t m = 0;
    for (uint32_t v : vmax_recent) m = v > m ? v : m;
    return m;
  }
  uint32_t recent_nmax() const {
    uint32_t m = 0;
    for (uint32_t v : nmax_recent) m = v > m ? v : m;
    return m;
  }
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  DevBuf<uint8_t> vec;
  DevBuf<uint32_t> adj0, uid, up_base, adjU, inv_uid;
  // search scratch: the handle's own stream, then caller streams of the device API
  Scratch main;
  std::vector<std::pair<hipStream_t, std::unique_ptr<Scratch>>> by_stream;
  // staging sets of the host-pointer API (HostStage), free for the next call
  std::vector<std::unique_ptr<HostStage>> stages_free;
  // the host-pointer API's own in-flight streams: a call's chunks (shine_knn_batch, kHostChunk queries) go round-robin
  // over them, after whatever the slot's own stream held when the call was enqueued (the fork event)
  std::vector<hipStream_t> hstreams;
  uint64_t hnext = 0;  // the host stream an asynchronous call's first chunk takes
  hipEvent_t hfork = nullptr;
  DevBuf<unsigned long long> prof;  // SHINE_PHASE_PROFILE diagnostics
  // dynamic record cache (SHINE_CACHE_DYNAMIC): this GPU's arena, lookup table, logs and the host policy engine
  DevBuf<uint32_t> cslot, cbits, cool, rlog, rlogged, slot_id, logn, upd;
  DevBuf<uint8_t> cvec;
  DevBuf<unsigned long long> clog;
  uint32_t clog_cap = 0, rlog_cap = 0, dyn_call = 0;
  uint32_t log_epoch = 0;  // advanced every time the logs are fetched and zeroed (DevGraph::dyn_epoch)
  RecordCache cache;
  // the policy's pipeline (capi.cc): logs of past calls copied to the host and not replayed yet; the arena updates a
  // replay made, not uploaded yet; a device-API search ran on another stream since the last update
  std::vector<unsigned long long> pend_clog;
  std::vector<uint32_t> pend_rlog;
  uint64_t pend_lost = 0;  // log entries past the device logs' capacity
  // the logs a replay works on (moved out of pend_* as it starts: the next call's logs are fetched while it runs)
  std::vector<unsigned long long> rp_clog;
  std::vector<uint32_t> rp_rlog;
  uint64_t rp_lost = 0;
  bool dyn_full = false;  // the engine's full() after its last finished replay (read by launches while one runs)
  std::vector<uint32_t> upd_vec;
  uint32_t upd_drop = 0, upd_fill = 0, upd_cool = 0;
  HostBuf<uint32_t> logn_h, rlog_h;  // pinned landing of the log counts and logs (copies of all slots in flight at once)
  bool counts_inflight = false;      // the counts' copy is enqueued behind this call's searches
  HostBuf<unsigned long long> clog_h;
  HostBuf<uint32_t> upd_host;
  bool dev_api_dirty = false;
  void release_dynamic() {
    for (auto* b : {&cslot, &cbits, &cool, &rlog, &rlogged, &slot_id, &logn, &upd}) b->release();
    cvec.release();
    clog.release();
    upd_host.release();
    logn_h.release();
    rlog_h.release();
    clog_h.release();
    clog_cap = rlog_cap = dyn_call = log_epoch = 0;
    counts_inflight = false;
    cache = RecordCache();
    pend_clog.clear();
    pend_rlog.clear();
    pend_lost = 0;
    rp_clog.clear();
    rp_rlog.clear();
    rp_lost = 0;
    dyn_full = false;
    upd_vec.clear();
    upd_drop = upd_fill = upd_cool = 0;
    dev_api_dirty = false;
  }
};

// Everything a handle holds but its lock: shine_cache_warmup builds a new layout into a second state and moves it in.
struct IndexState {
  uint32_t dim = 0, M = 0, M0 = 0;
  int metric = 0, elem = 0;
  uint64_t N = 0, upper_rows = 0;
  uint32_t ep = 0, ep_level = 0, ep_uid = 0, n_shards = 0, lists_unique = 1;
  uint32_t inv_size = 0;
  uint64_t words_per_slot = 0;
  uint64_t device_bytes = 0;
  int search_mode = SHINE_MODE_EXACT;
  int placement = SHINE_PLACE_REPLICA;
  uint64_t id_space = 0;       // device ids are < id_space (sharded: slot o owns [o * ids_per_slot, ...))
  uint64_t ids_per_slot = 0;
  uint64_t cached_rows = 0;    // sharded: vectors of every stripe other slots keep local copies of
  uint64_t cached_list_rows = 0;  // ... and neighbour lists (each array's copy is whole VM pages of that array)
  uint32_t div_magic = 0, div_shift = 0;  // id / ids_per_slot = umulhi(id, div_magic) >> div_shift
  ShardedArray svec, sadj0;    // sharded: level-0 vectors and lists
  double cache_fraction = 0;   // the cached share of every stripe's vectors, after rounding to whole pages
  double cache_requested = 0;  // the caller's cache_fraction (a re-layout after a warmup rounds it again)
  Regions regions;             // SHINE_PLACE_SHARDED_REGIONS: slot o owns (and is routed) region o
  Router router;               // ... the query router's limits and histogram, kept across calls
  std::vector<double> slot_rate;  // ... queries per ms each slot answered in its last call (0 = not measured)
  std::vector<Replica> reps;
  // sharded placements: the host graph and its device ids, kept to re-rank the stripes after a cache warmup
  HostGraph host;
  std::vector<uint32_t> dev_of;  // dev_of[g] = device id of graph node g
  std::vector<int> devs;
  // sharded placements: uid of every device id and device id of every uid (host copies, for the dynamic cache)
  std::vector<uint32_t> uid_of_dev, dev_of_uid;
  int cache_policy = SHINE_CACHE_STATIC;
  uint64_t cache_seed = 0;
  uint64_t cache_entries_per_gpu = 0;
};


// Search entry points of capi.cc for other translation units of the library (the GPU batch builder).
// Enqueue the pass chain of one batch on stream s (device pointers; asynchronous).
int search_enqueue(shine_index* h, uint32_t slot, const float* d_q, uint32_t nq, uint32_t k, uint32_t ef,
                   uint32_t* d_ids, float* d_dists, uint32_t* d_qs, hipStream_t s);
void index_release(shine_index* h);
// An index handle over a host graph (as shine_open_buffers_ex builds one from parsed dumps).
int index_from_graph(HostGraph&& G, int elem, const int* gpu_ids, uint32_t n_gpus, int placement, double cache_fraction,
                     shine_index_t* out);

}  // namespace shine

namespace shine {

// Worker threads kept for the handle's lifetime (the dynamic cache's per-slot replays between calls): spawning a
// thread per slot and call cost ~0.1-0.3 ms of a 4 ms call.
class TaskPool {
 public:
  TaskPool() = default;
  TaskPool(const TaskPool&) = delete;
  TaskPool& operator=(const TaskPool&) = delete;
  ~TaskPool() {
    wait();
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    go_.notify_all();
    for (auto& t : th_) t.join();
  }
  // f(i) for every i < n, on up to n - 1 pool threads and the caller's; returns when all are done
  void run(size_t n, const std::function<void(size_t)>& f) {
    if (n == 0) return;
    wait();  // (a launch still running)
    {
      std::lock_guard<std::mutex> lk(m_);
      // a new worker starts from the current generation, so it joins this run, not a finished one
      while (th_.size() + 1 < n) th_.emplace_back([this, g = gen_] { worker(g); });
      f_ = &f;
      n_ = n;
      next_ = 0;
      active_ = th_.size();
      ++gen_;
    }
    go_.notify_all();
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return active_ == 0; });
    f_ = nullptr;
  }
  // f(i) for every i < n on n pool threads, returning at once (the caller takes no share); wait() joins it
  void launch(size_t n, std::function<void(size_t)> f) {
    if (n == 0) return;
    wait();
    {
      std::lock_guard<std::mutex> lk(m_);
      while (th_.size() < n) th_.emplace_back([this, g = gen_] { worker(g); });
      own_ = std::move(f);
      f_ = &own_;
      n_ = n;
      next_ = 0;
      active_ = th_.size();
      ++gen_;
    }
    go_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return active_ == 0; });
    f_ = nullptr;
  }

 private:
  void worker(uint64_t seen) {
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      go_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(size_t)>* f = f_;
      const size_t n = n_;
      lk.unlock();
      for (size_t i; (i = next_.fetch_add(1)) < n;) (*f)(i);
      lk.lock();
      if (--active_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable go_, done_;
  const std::function<void(size_t)>* f_ = nullptr;
  std::function<void(size_t)> own_;  // a launch's function
  size_t n_ = 0, active_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace shine

// The opaque handle of include/shine_gpu.h.
struct shine_index : shine::IndexState {
  std::vector<shine_request*> requests;  // shine_knn_batch_async calls not waited for yet
  // the dynamic cache's replay running on the pool past a host call's return (capi.cc replay_launch / wait_replay),
  // its per-slot statistics, and those of finished replays no call has reported yet
  bool replay_busy = false;
  std::vector<shine_stats> replay_per, replay_unreported;
  std::mutex mu;
  shine::TaskPool pool;  // (declared last: its threads stop before the state they work on goes)
};
