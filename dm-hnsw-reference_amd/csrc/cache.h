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

// A zero-filled array in its own mapping, backed by 2 MiB pages where the kernel allows (madvise): the policy's random
// picks over tens of MiB of bucket records otherwise pay a TLB miss and a page walk on top of each cache miss.
template <typename T>
class HugeArray {
 public:
  HugeArray() = default;
  explicit HugeArray(size_t n);
  HugeArray(HugeArray&& o) noexcept : p_(o.p_), n_(o.n_), bytes_(o.bytes_) { o.p_ = nullptr; o.n_ = o.bytes_ = 0; }
  HugeArray& operator=(HugeArray&& o) noexcept {
    if (this != &o) {
      release();
      p_ = o.p_; n_ = o.n_; bytes_ = o.bytes_;
      o.p_ = nullptr; o.n_ = o.bytes_ = 0;
    }
    return *this;
  }
  HugeArray(const HugeArray&) = delete;
  HugeArray& operator=(const HugeArray&) = delete;
  ~HugeArray() { release(); }
  T* data() { return p_; }
  const T* data() const { return p_; }
  size_t size() const { return n_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }

 private:
  void release();
  T* p_ = nullptr;
  size_t n_ = 0, bytes_ = 0;
};

// x % d for a fixed d by multiplication (Lemire, Kaser, Kurz, "Faster remainder by direct computation", 2019: a
// 128-bit reciprocal, exact for every 64-bit x and d): the policy takes several remainders per step (bucket of a key,
// cooling bucket, random pick), and a 64-bit divide costs tens of cycles each.
struct FastMod {
  unsigned __int128 m = 0;
  uint64_t d = 1;
  FastMod() = default;
  explicit FastMod(uint64_t div) : m(~static_cast<unsigned __int128>(0) / div + 1), d(div) {}
  uint64_t operator()(uint64_t x) const {
    const unsigned __int128 low = m * x;
    const unsigned __int128 bottom = (static_cast<unsigned __int128>(static_cast<uint64_t>(low)) * d) >> 64;
    const unsigned __int128 top = static_cast<unsigned __int128>(static_cast<uint64_t>(low >> 64)) * d;
    return static_cast<uint64_t>((bottom + top) >> 64);
  }
};

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
  // key_space: keys are below it (record uids)
  RecordCache(uint32_t entries, uint64_t seed, uint32_t key_space);

  uint32_t capacity() const { return C_; }
  // evict() terminates only if the cache holds more entries than its cooling table (6 per bucket): otherwise every
  // entry can end up cooling with no bucket full, and the reference's loop never finds a victim (cache.hh:232-311)
  static bool size_ok(uint32_t entries);
  bool full() const { return next_idx_ >= C_; }  // cache.hh:205-216
  bool contains(uint32_t key) const { return slot_of(key) != 0xFFFFFFFFu; }

  // The policy over one call's logs.  rescued: keys of the cooling entries hit; candidates: the misses offered.
  // Appends the arena changes to `updates` and to `flagged` the slots whose cooling flag changed (set by the eviction
  // scan, cleared by a second chance); slots whose entry left the cache are reported in updates (their flag is cleared
  // with the copy).
  void apply_call(std::vector<uint32_t> rescued, std::vector<CacheCandidate> candidates,
                  std::vector<CacheUpdate>& updates, std::vector<uint32_t>& flagged);

  std::vector<uint32_t> keys() const;
  uint32_t slot_key(uint32_t slot) const { return slot < key_of_.size() ? key_of_[slot] : 0xFFFFFFFFu; }
  uint32_t slot_of(uint32_t key) const;
  bool cooling(uint32_t slot) const { return slot < cooling_.size() && cooling_[slot] != 0; }

  uint64_t admitted = 0, evicted = 0, rescued = 0;
  // diagnostics of the last apply_call (SHINE_DEBUG_CACHE_TIMING): eviction-scan steps, and the ms of its second
  // chances, of the candidates' sort and of the admissions
  uint64_t scan_steps = 0;
  double ms_rescue = 0, ms_sort = 0, ms_admit = 0;

 private:
  // A draw of the stream with what the scan derives from it, computed when it enters the ring (kAhead draws before it
  // is taken, off the scan's chain of dependent steps): the bucket it picks (v % B) and v % 60, which gives the pick of
  // an entry in a bucket of n <= 5 entries as (v % 60) % n (every such n divides 60) by a table read.
  struct Draw {
    uint64_t v;
    uint32_t b;
    uint32_t r60;
  };
  Draw rand();                        // the next draw of the stream
  const Draw& peek(uint32_t i) const; // the draw i ahead (1 <= i <= kAhead), not taken
  uint64_t next_draw();               // SplitMix64 step: the draw kAhead ahead of rand()'s
  void push_draw(uint32_t slot);      // ring slot <- the next draw, its bucket requested
  uint32_t pick(const Draw& d, uint32_t n) const {  // d.v % n, the entry a draw picks in a bucket of n
    return n <= kInPlace ? kPick60[d.r60][n] : static_cast<uint32_t>(d.v % n);
  }
  uint32_t cool_bucket(uint32_t key) {  // cool_of(key), from the look-ahead's memo when it computed it
    return key == memo_key_ ? memo_cool_ : cool_of(key);
  }
  struct Victim {
    uint32_t slot, dev;
  };
  Victim evict();  // cache.hh:232-311: frees one slot (and names the device id that leaves it)
  void lookahead();
  void insert(uint32_t key, uint32_t dev, std::vector<CacheUpdate>& updates);
  bool ct_remove(uint32_t key);
  // key (home bucket b, cooling bucket c) in; when the cooling bucket was full its oldest key leaves: victim, vbucket
  bool ct_insert(uint32_t key, uint32_t b, uint32_t c, uint32_t& victim, uint32_t& vbucket);

  // Hash buckets as flat 64-byte records, one cache line each: [count | cooling bits << 16, (key, slot, device id) x 5]
  // in insertion order.  A lookup, the eviction scan's random pick with its cooling flag, and an erase with the
  // leaving device id each touch that one line: no key -> slot array, no slot -> flag or slot -> device read on the
  // scan's path (the policy is a chain of dependent misses; each array read on it was one more).  A bucket holds 5
  // entries in place and the rare rest (Poisson(1) occupancy: ~6e-4 of the buckets) in `bover_` as (key, slot,
  // device, cooling) in order.  The slot arrays below are written on the way for the callers' per-slot reads.
  // Cooling-table buckets: 16-word records [count, up to 6 keys newest first, their hash buckets in the same order]:
  // the key a full bucket pushes out comes with its hash bucket, so the scan reads the victim's record without hashing
  // it first (and the look-ahead requests that record one step early).
  static constexpr uint32_t kBW = 16, kInPlace = 5, kCW = 16, kCB = 7;
  static const uint8_t (&kPick60)[60][kInPlace + 1];  // [v % 60][n] = v % n
  struct Ent {
    uint32_t key, slot, dev;
    bool cool;
  };
  uint32_t* brec(uint32_t b) { return bk_.data() + static_cast<size_t>(b) * kBW; }
  const uint32_t* brec(uint32_t b) const { return bk_.data() + static_cast<size_t>(b) * kBW; }
  static uint32_t bcount(const uint32_t* r) { return r[0] & 0xFFFFu; }
  uint32_t bucket_of(uint32_t key) const;
  uint32_t cool_of(uint32_t key) const;  // the key's cooling-table bucket
  int bfind(uint32_t b, uint32_t key, Ent& e) const;  // the key's position in bucket b (its entry in e), or -1
  Ent bget(uint32_t b, uint32_t i) const;
  void bset_cool(uint32_t b, uint32_t i, bool cool);
  void bpush(uint32_t b, uint32_t key, uint32_t slot, uint32_t dev);
  void berase(uint32_t b, uint32_t i);  // entry i out, the others in order (vector::erase in the reference's Bucket)

  uint32_t C_ = 0, B_ = 1, CT_ = 1, next_idx_ = 0, key_space_ = 0;
  FastMod modB_, modCT_, mod60_;  // % B_, % CT_, % 60
  uint64_t state_ = 0;
  // the next kAhead draws, computed once each with their hash bucket (a draw picks a bucket, or an entry of one): each
  // bucket is requested kAhead draws before the eviction scan may read it
  static constexpr uint32_t kAhead = 8;
  Draw ring_[kAhead] = {};
  uint32_t head_ = 0;
  uint32_t memo_key_ = 0xFFFFFFFFu, memo_cool_ = 0;  // the look-ahead's cool_of(memo_key_)
  HugeArray<uint32_t> bk_;  // [B_][kBW] (page-aligned: records on cache-line boundaries)
  std::unordered_map<uint32_t, std::vector<uint32_t>> bover_;  // bucket -> (key, slot, dev, cool) past kInPlace
  HugeArray<uint32_t> ct_;                                     // [CT_][kCW]
  HugeArray<uint32_t> key_of_, dev_of_;                        // slot -> key / device id
  HugeArray<uint8_t> cooling_;                                 // slot -> cooling
  std::vector<uint32_t>* flagged_ = nullptr;
};

// entries of a compute node's cache: ratio % of estimate_index_size(n) over the record prefix size 16 + 4d
// (compute_node.cc:40-56, hnsw.hh:309-321)
uint64_t cache_entries(uint64_t n, uint32_t M, uint32_t dim, double ratio_percent);

}  // namespace shine
