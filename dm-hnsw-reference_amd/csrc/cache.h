// Host engine of the dynamic record cache (SHINE_CACHE_DYNAMIC): the reference's compute-node cache::Cache
// (src/cache/cache.hh:24-311) with its CoolingTable (cooling_table.hh:52-98), applied between calls.
//
// During a call the cache of a GPU is fixed: the kernels read cached records from the GPU's arena and log the
// misses offered for admission and the cooling entries they hit (kernels.h DevGraph::cslot / clog / rlog).  After the
// call this engine replays the reference's policy over those logs — second chances first, then admissions in
// (query, key) order — and returns the arena updates (records to copy in, keys to drop, cooling flags to set).
// Keys are record uids.  The reference seeds its random draws from std::random_device; one SplitMix64 stream per
// cache (seeded) drives them here, so a run is reproducible and oracle/cache_ref.py, an independent restatement,
// predicts every hit count and the cache contents after every call.
#pragma once

#include <cstdint>
#include <unordered_map>
#include <vector>

namespace shine {

struct CacheCandidate {
  uint32_t query, key;  // query index of the call, record uid
  uint32_t dev_id;      // the record's device id
  bool always, coin;    // admitted without the coin (entry point, upper levels) / the coin passed
};

struct CacheUpdate {
  uint32_t slot;        // arena slot
  uint32_t new_dev;     // device id now cached in the slot (copy its row in)
  uint32_t old_dev;     // device id that left the slot (0xFFFFFFFF: the slot was free)
};

class RecordCache {
 public:
  RecordCache() = default;
  // key_space: keys are below it (record uids; the key -> slot map is a flat array of that many entries)
  RecordCache(uint32_t entries, uint64_t seed, uint32_t key_space);

  uint32_t capacity() const { return C_; }
  // evict() terminates only if the cache holds more entries than its cooling table (6 per bucket): otherwise every
  // entry can end up cooling with no bucket full, and the reference's loop never finds a victim (cache.hh:232-311)
  static bool size_ok(uint32_t entries);
  bool full() const { return next_idx_ >= C_; }  // cache.hh:205-216
  bool contains(uint32_t key) const { return key < slot_of_.size() && slot_of_[key] != 0xFFFFFFFFu; }

  // The policy over one call's logs.  rescued: keys of the cooling entries hit; candidates: the misses offered.
  // Appends the arena changes to `updates` and the slots whose cooling flag must be set to `cool_on`; slots whose
  // entry left the cache are reported in updates (their flag is cleared with the copy).
  void apply_call(std::vector<uint32_t> rescued, std::vector<CacheCandidate> candidates,
                  std::vector<CacheUpdate>& updates, std::vector<uint32_t>& cool_on);

  std::vector<uint32_t> keys() const;
  uint32_t slot_key(uint32_t slot) const { return slot < key_of_.size() ? key_of_[slot] : 0xFFFFFFFFu; }
  uint32_t slot_of(uint32_t key) const { return contains(key) ? slot_of_[key] : 0xFFFFFFFFu; }
  bool cooling(uint32_t slot) const { return slot < cooling_.size() && cooling_[slot] != 0; }

  uint64_t admitted = 0, evicted = 0, rescued = 0;

 private:
  uint64_t rand();
  uint64_t peek(uint32_t i) const;
  uint32_t evict();  // cache.hh:232-311: frees one slot
  void insert(uint32_t key, uint32_t dev, std::vector<CacheUpdate>& updates);
  bool ct_remove(uint32_t key);
  bool ct_insert(uint32_t key, uint32_t& victim);

  // Hash buckets (keys in insertion order) and cooling-table buckets (newest first) as flat arrays of 8-word records:
  // [count, entries...] — the policy's random picks land on a bucket in one cache line instead of a vector header and
  // its heap block (two misses; the replay of a full cache spent ~1.5 us per admission there).  A hash bucket holds 7
  // entries in place and the rare rest (Poisson(1) occupancy: ~1e-5 of the buckets) in `bover_`, in order.
  static constexpr uint32_t kBW = 8, kInPlace = 7;
  uint32_t bsize(uint32_t b) const { return bk_[static_cast<size_t>(b) * kBW]; }
  uint32_t bget(uint32_t b, uint32_t i) const;
  void bpush(uint32_t b, uint32_t key);
  void berase(uint32_t b, uint32_t key);

  uint32_t C_ = 0, B_ = 1, CT_ = 1, next_idx_ = 0;
  uint64_t state_ = 0;
  std::vector<uint32_t> bk_;                                   // [B_][kBW]
  std::unordered_map<uint32_t, std::vector<uint32_t>> bover_;  // bucket -> entries past kInPlace
  std::vector<uint32_t> ct_;                                   // [CT_][kBW]: count, up to 6 keys newest first
  std::vector<uint32_t> slot_of_;                   // key -> arena slot (0xFFFFFFFF: not cached)
  std::vector<uint32_t> key_of_, dev_of_;           // slot -> key / device id
  std::vector<uint8_t> cooling_;                    // slot -> cooling
  std::vector<uint32_t>* cool_on_ = nullptr;
};

// entries of a compute node's cache: ratio % of estimate_index_size(n) over the record prefix size 16 + 4d
// (compute_node.cc:40-56, hnsw.hh:309-321)
uint64_t cache_entries(uint64_t n, uint32_t M, uint32_t dim, double ratio_percent);

}  // namespace shine
