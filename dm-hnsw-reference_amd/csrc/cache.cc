// Dynamic record cache engine: cache::Cache + CoolingTable (src/cache/cache.hh:24-311, cooling_table.hh:52-98) at
// call granularity.  See cache.h.
#include "cache.h"

#include <sys/mman.h>

#include <algorithm>
#include <cmath>
#include <new>
#ifndef SHINE_CACHE_PF
#define SHINE_CACHE_PF 4
#endif

namespace shine {

namespace {

constexpr uint32_t kInv = 0xFFFFFFFFu;
constexpr uint32_t kCoolingBucketEntries = 6;  // constants.hh:14
constexpr double kCoolingRatio = 0.1;          // constants.hh:15

uint64_t murmur64(uint64_t h) {  // std::hash<RemotePtr> (remote_pointer.hh:31-51) over the key
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

uint64_t splitmix(uint64_t z) {  // the cooling table's hash (cooling_table.hh:100-108)
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

uint64_t cache_entries(uint64_t n, uint32_t M, uint32_t dim, double ratio_percent) {
  if (n == 0 || M < 2) return 0;
  const uint32_t levels = static_cast<uint32_t>(std::round(std::log(static_cast<double>(n)) / std::log(M)));
  uint64_t index_size = 0;  // hnsw.hh:309-321
  for (uint32_t i = 0; i < levels; ++i) {
    const uint64_t size = i == 0 ? (16ull + 4ull * dim) + (4ull + 8ull * 2 * M) : 4ull + 8ull * M;
    index_size += static_cast<uint64_t>(std::llround(std::pow(1.0 / M, i) * static_cast<double>(n))) * size;
  }
  // static_cast<f32>(estimated_index_size) / 100. * ratio, in double after the f32 rounding (compute_node.cc:43)
  const uint64_t cache_size =
      static_cast<uint64_t>(static_cast<double>(static_cast<float>(index_size)) / 100. * ratio_percent);
  return cache_size / (16ull + 4ull * dim);  // compute_node.cc:40-54
}

template <typename T>
HugeArray<T>::HugeArray(size_t n) : n_(n) {
  if (n == 0) return;
  constexpr size_t kHuge = 2u << 20;
  bytes_ = (n * sizeof(T) + kHuge - 1) / kHuge * kHuge;
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  madvise(p, bytes_, MADV_HUGEPAGE);  // a hint: without huge pages the array still works (zero-filled by mmap)
  p_ = static_cast<T*>(p);
}

template <typename T>
void HugeArray<T>::release() {
  if (p_) munmap(p_, bytes_);
  p_ = nullptr;
  n_ = bytes_ = 0;
}

template class HugeArray<uint32_t>;
template class HugeArray<uint8_t>;

RecordCache::RecordCache(uint32_t entries, uint64_t seed, uint32_t key_space)
    : C_(entries),
      B_(std::max<uint32_t>(1, entries)),
      CT_(std::max<uint32_t>(1, static_cast<uint32_t>(std::ceil(entries / static_cast<double>(kCoolingBucketEntries) *
                                                                kCoolingRatio)))),
      key_space_(key_space),
      state_(seed),
      bk_(static_cast<size_t>(B_) * kBW),
      ct_(static_cast<size_t>(CT_) * kCW),
      key_of_(entries),
      dev_of_(entries),
      cooling_(entries) {
  modB_ = FastMod(B_);
  modCT_ = FastMod(CT_);
  for (uint32_t n = 1; n <= kInPlace; ++n) mod_n_[n] = FastMod(n);
  std::fill(key_of_.data(), key_of_.data() + entries, kInv);
  std::fill(dev_of_.data(), dev_of_.data() + entries, kInv);
}

bool RecordCache::size_ok(uint32_t entries) {
  const uint32_t ct = std::max<uint32_t>(
      1, static_cast<uint32_t>(std::ceil(entries / static_cast<double>(kCoolingBucketEntries) * kCoolingRatio)));
  return entries > kCoolingBucketEntries * ct;
}

uint64_t RecordCache::rand() {
  state_ += 0x9E3779B97F4A7C15ull;
  uint64_t z = state_;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint32_t RecordCache::bucket_of(uint32_t key) const { return static_cast<uint32_t>(modB_(murmur64(key))); }
uint32_t RecordCache::cool_of(uint32_t key) const { return static_cast<uint32_t>(modCT_(splitmix(key))); }

uint32_t RecordCache::bfind(uint32_t b, uint32_t key) const {
  const uint32_t* r = brec(b);
  const uint32_t in = r[0] < kInPlace ? r[0] : kInPlace;
  for (uint32_t i = 0; i < in; ++i)
    if (r[1 + 2 * i] == key) return r[2 + 2 * i];
  if (r[0] > kInPlace) {
    const std::vector<uint32_t>& o = bover_.at(b);
    for (size_t i = 0; i < o.size(); i += 2)
      if (o[i] == key) return o[i + 1];
  }
  return kInv;
}

uint32_t RecordCache::slot_of(uint32_t key) const {
  if (C_ == 0 || key >= key_space_) return kInv;
  return bfind(bucket_of(key), key);
}

void RecordCache::bget(uint32_t b, uint32_t i, uint32_t& key, uint32_t& slot) const {
  if (i < kInPlace) {
    key = brec(b)[1 + 2 * i];
    slot = brec(b)[2 + 2 * i];
    return;
  }
  const std::vector<uint32_t>& o = bover_.at(b);
  key = o[2 * (i - kInPlace)];
  slot = o[2 * (i - kInPlace) + 1];
}

void RecordCache::bpush(uint32_t b, uint32_t key, uint32_t slot) {
  uint32_t* r = brec(b);
  if (r[0] < kInPlace) {
    r[1 + 2 * r[0]] = key;
    r[2 + 2 * r[0]] = slot;
  } else {
    auto& o = bover_[b];
    o.push_back(key);
    o.push_back(slot);
  }
  ++r[0];
}

// remove key from bucket b, keeping the others in order (vector::erase in the reference's Bucket)
void RecordCache::berase(uint32_t b, uint32_t key) {
  uint32_t* r = brec(b);
  const uint32_t n = r[0];
  const uint32_t in = n < kInPlace ? n : kInPlace;
  uint32_t i = 0;
  while (i < in && r[1 + 2 * i] != key) ++i;
  if (i < in) {
    for (uint32_t j = i; j + 1 < in; ++j) {
      r[1 + 2 * j] = r[3 + 2 * j];
      r[2 + 2 * j] = r[4 + 2 * j];
    }
    if (n > kInPlace) {  // the first entry past the in-place ones moves in
      auto it = bover_.find(b);
      r[1 + 2 * (kInPlace - 1)] = it->second[0];
      r[2 + 2 * (kInPlace - 1)] = it->second[1];
      it->second.erase(it->second.begin(), it->second.begin() + 2);
      if (it->second.empty()) bover_.erase(it);
    }
  } else {
    auto it = bover_.find(b);
    auto& o = it->second;
    size_t k = 0;
    while (o[k] != key) k += 2;
    o.erase(o.begin() + k, o.begin() + k + 2);
    if (o.empty()) bover_.erase(it);
  }
  r[0] = n - 1;
}

bool RecordCache::ct_remove(uint32_t key) {  // cooling_table.hh:52-75
  uint32_t* r = &ct_[static_cast<size_t>(cool_of(key)) * kCW];
  uint32_t i = 0;
  while (i < r[0] && r[1 + i] != key) ++i;
  if (i == r[0]) return false;
  for (uint32_t j = i; j + 1 < r[0]; ++j) r[1 + j] = r[2 + j];
  --r[0];
  return true;
}

bool RecordCache::ct_insert(uint32_t key, uint32_t& victim) {  // cooling_table.hh:81-98
  uint32_t* r = &ct_[static_cast<size_t>(cool_of(key)) * kCW];
  bool pushed = false;
  if (r[0] == kCoolingBucketEntries) {  // the oldest (last) key leaves
    victim = r[kCoolingBucketEntries];
    --r[0];
    pushed = true;
  }
  for (uint32_t j = r[0]; j > 0; --j) r[1 + j] = r[j];  // newest first
  r[1] = key;
  ++r[0];
  return pushed;
}

// The draw i ahead of the stream without taking it (prefetch hints only).
uint64_t RecordCache::peek(uint32_t i) const {
  uint64_t z = state_ + 0x9E3779B97F4A7C15ull * i;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// The next pick of the eviction scan, read ahead (its bucket's line was requested SHINE_CACHE_PF draws earlier): the
// lines its step will touch — the entry's cooling flag, its cooling-table bucket and, when that bucket is full, the
// hash bucket of the key it would push out — are requested now, so that the victim lookup, the scan's one dependent
// miss, overlaps this step's.  A hint only: the step itself re-reads everything.
void RecordCache::lookahead() const {
  const uint32_t* r = brec(static_cast<uint32_t>(modB_(peek(1))));
  const uint32_t n = r[0];
  if (n == 0 || n > kInPlace) return;
  const uint32_t i = static_cast<uint32_t>(mod_n_[n](peek(2)));
  const uint32_t key = r[1 + 2 * i];
  __builtin_prefetch(&cooling_[r[2 + 2 * i]]);
  const uint32_t* c = &ct_[static_cast<size_t>(cool_of(key)) * kCW];
  if (c[0] == kCoolingBucketEntries) __builtin_prefetch(brec(bucket_of(c[kCoolingBucketEntries])));
}

uint32_t RecordCache::evict() {  // cache.hh:232-311
  for (;;) {
    const uint32_t b = static_cast<uint32_t>(modB_(rand()));
    // the next pick's bucket is one or two draws ahead (an empty bucket takes no entry draw): both requested now, so
    // the loop's dependent misses overlap
    for (uint32_t a = 1; a <= SHINE_CACHE_PF; ++a) __builtin_prefetch(brec(static_cast<uint32_t>(modB_(peek(a)))));
    const uint32_t n = brec(b)[0];
    if (n == 0) continue;
    uint32_t key, slot;
    bget(b, static_cast<uint32_t>(n <= kInPlace ? mod_n_[n](rand()) : rand() % n), key, slot);
    lookahead();
    uint32_t victim = kInv;
    bool has_victim = false;
    if (!cooling_[slot]) {  // hot -> cooling; the table may push its oldest key out
      has_victim = ct_insert(key, victim);
      cooling_[slot] = 1;
      if (flagged_) flagged_->push_back(slot);
    }
    if (!has_victim) continue;
    const uint32_t vb = bucket_of(victim);
    const uint32_t vslot = bfind(vb, victim);
    if (vslot == kInv || !cooling_[vslot]) continue;  // rescued meanwhile: no eviction
    berase(vb, victim);
    cooling_[vslot] = 0;
    ++evicted;
    return vslot;
  }
}

void RecordCache::insert(uint32_t key, uint32_t dev, std::vector<CacheUpdate>& updates) {  // cache.hh:147-203
  const uint32_t slot = next_idx_ < C_ ? next_idx_++ : evict();
  updates.push_back({slot, dev, dev_of_[slot]});
  bpush(bucket_of(key), key, slot);
  key_of_[slot] = key;
  dev_of_[slot] = dev;
  cooling_[slot] = 0;
  ++admitted;
}

// (query, key) order of the candidates: an LSD radix sort over the composite (query << 32 | key), 11-bit digits, only
// the digits the largest composite needs (a comparison sort of the ~340K candidates one slot logs while its cache
// fills took most of the time between calls)
void sort_candidates(std::vector<CacheCandidate>& c) {
  const size_t n = c.size();
  if (n < 2) return;
  std::vector<uint64_t> k(n), k2(n);
  std::vector<uint32_t> ix(n), ix2(n);
  uint64_t most = 0;
  for (size_t i = 0; i < n; ++i) {
    k[i] = (static_cast<uint64_t>(c[i].query) << 32) | c[i].key;
    ix[i] = static_cast<uint32_t>(i);
    most |= k[i];
  }
  constexpr int kDigit = 11;  // 2K counters a pass: a call's few thousand candidates take 4 cheap passes
  std::vector<uint32_t> cnt(1u << kDigit);
  for (int shift = 0; shift < 64 && (most >> shift) != 0; shift += kDigit) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    for (size_t i = 0; i < n; ++i) ++cnt[(k[i] >> shift) & ((1u << kDigit) - 1)];
    uint32_t sum = 0;
    for (uint32_t& x : cnt) {
      const uint32_t t = x;
      x = sum;
      sum += t;
    }
    for (size_t i = 0; i < n; ++i) {
      const uint32_t pos = cnt[(k[i] >> shift) & ((1u << kDigit) - 1)]++;
      k2[pos] = k[i];
      ix2[pos] = ix[i];
    }
    k.swap(k2);
    ix.swap(ix2);
  }
  std::vector<CacheCandidate> out(n);
  for (size_t i = 0; i < n; ++i) out[i] = c[ix[i]];
  c.swap(out);
}

void RecordCache::apply_call(std::vector<uint32_t> rescued_keys, std::vector<CacheCandidate> candidates,
                             std::vector<CacheUpdate>& updates, std::vector<uint32_t>& flagged) {
  if (C_ == 0) return;
  flagged_ = &flagged;
  std::sort(rescued_keys.begin(), rescued_keys.end());
  rescued_keys.erase(std::unique(rescued_keys.begin(), rescued_keys.end()), rescued_keys.end());
  constexpr size_t kAhead = 8;  // lookups requested this many keys ahead (each one a likely miss)
  const size_t nr = rescued_keys.size();
  for (size_t i = 0; i < nr; ++i) {  // cache.hh:128-132
    if (i + kAhead < nr && rescued_keys[i + kAhead] < key_space_) {
      const uint32_t k = rescued_keys[i + kAhead];
      __builtin_prefetch(brec(bucket_of(k)));
      __builtin_prefetch(&ct_[static_cast<size_t>(cool_of(k)) * kCW]);
    }
    const uint32_t key = rescued_keys[i];
    const uint32_t slot = slot_of(key);
    if (slot != kInv && cooling_[slot] && ct_remove(key)) {
      cooling_[slot] = 0;
      flagged.push_back(slot);
      ++rescued;
    }
  }
  sort_candidates(candidates);  // (query, key): a query offers a key once, so the order is total
  const size_t nc = candidates.size();
  for (size_t i = 0; i < nc; ++i) {
    if (i + kAhead < nc && candidates[i + kAhead].key < key_space_)
      __builtin_prefetch(brec(bucket_of(candidates[i + kAhead].key)));
    const CacheCandidate& c = candidates[i];
    if (c.key >= key_space_ || contains(c.key)) continue;  // admitted by an earlier miss (cache.hh:171-179)
    if (c.always || !full() || c.coin) insert(c.key, c.dev_id, updates);
  }
  flagged_ = nullptr;
}

std::vector<uint32_t> RecordCache::keys() const {
  std::vector<uint32_t> out;
  for (size_t s = 0; s < key_of_.size(); ++s)
    if (const uint32_t k = key_of_[s]; k != kInv && slot_of(k) == s) out.push_back(k);
  std::sort(out.begin(), out.end());
  return out;
}

}  // namespace shine
