// Dynamic record cache engine: cache::Cache + CoolingTable (src/cache/cache.hh:24-311, cooling_table.hh:52-98) at
// call granularity.  See cache.h.
#include "cache.h"

#include <algorithm>
#include <cmath>

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

RecordCache::RecordCache(uint32_t entries, uint64_t seed, uint32_t key_space)
    : C_(entries),
      B_(std::max<uint32_t>(1, entries)),
      CT_(std::max<uint32_t>(1, static_cast<uint32_t>(std::ceil(entries / static_cast<double>(kCoolingBucketEntries) *
                                                                kCoolingRatio)))),
      state_(seed),
      bk_(static_cast<size_t>(B_) * kBW, 0),
      ct_(static_cast<size_t>(CT_) * kBW, 0),
      key_of_(entries, kInv),
      dev_of_(entries, kInv),
      cooling_(entries, 0) {
  slot_of_.assign(key_space, kInv);
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

uint32_t RecordCache::bget(uint32_t b, uint32_t i) const {
  if (i < kInPlace) return bk_[static_cast<size_t>(b) * kBW + 1 + i];
  return bover_.at(b)[i - kInPlace];
}

void RecordCache::bpush(uint32_t b, uint32_t key) {
  uint32_t* r = &bk_[static_cast<size_t>(b) * kBW];
  if (r[0] < kInPlace) r[1 + r[0]] = key;
  else bover_[b].push_back(key);
  ++r[0];
}

// remove key from bucket b, keeping the others in order (vector::erase in the reference's Bucket)
void RecordCache::berase(uint32_t b, uint32_t key) {
  uint32_t* r = &bk_[static_cast<size_t>(b) * kBW];
  const uint32_t n = r[0];
  const uint32_t in = n < kInPlace ? n : kInPlace;
  uint32_t i = 0;
  while (i < in && r[1 + i] != key) ++i;
  if (i < in) {
    for (uint32_t j = i; j + 1 < in; ++j) r[1 + j] = r[2 + j];
    if (n > kInPlace) {  // the first entry past the in-place ones moves in
      auto it = bover_.find(b);
      r[kInPlace] = it->second.front();
      it->second.erase(it->second.begin());
      if (it->second.empty()) bover_.erase(it);
    }
  } else {
    auto it = bover_.find(b);
    it->second.erase(std::find(it->second.begin(), it->second.end(), key));
    if (it->second.empty()) bover_.erase(it);
  }
  r[0] = n - 1;
}

bool RecordCache::ct_remove(uint32_t key) {  // cooling_table.hh:52-75
  uint32_t* r = &ct_[static_cast<size_t>(splitmix(key) % CT_) * kBW];
  uint32_t i = 0;
  while (i < r[0] && r[1 + i] != key) ++i;
  if (i == r[0]) return false;
  for (uint32_t j = i; j + 1 < r[0]; ++j) r[1 + j] = r[2 + j];
  --r[0];
  return true;
}

bool RecordCache::ct_insert(uint32_t key, uint32_t& victim) {  // cooling_table.hh:81-98
  uint32_t* r = &ct_[static_cast<size_t>(splitmix(key) % CT_) * kBW];
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

uint32_t RecordCache::evict() {  // cache.hh:232-311
  for (;;) {
    const uint32_t b = static_cast<uint32_t>(rand() % B_);
    // the next pick's bucket is one or two draws ahead (an empty bucket takes no entry draw): both requested now, so
    // the loop's dependent misses overlap (an admission into a full cache took ~1 us of misses)
    __builtin_prefetch(&bk_[static_cast<size_t>(peek(1) % B_) * kBW]);
    __builtin_prefetch(&bk_[static_cast<size_t>(peek(2) % B_) * kBW]);
    const uint32_t n = bsize(b);
    if (n == 0) continue;
    const uint32_t key = bget(b, static_cast<uint32_t>(rand() % n));
    const uint32_t slot = slot_of_[key];
    uint32_t victim = kInv;
    bool has_victim = false;
    if (!cooling_[slot]) {  // hot -> cooling; the table may push its oldest key out
      has_victim = ct_insert(key, victim);
      cooling_[slot] = 1;
      if (cool_on_) cool_on_->push_back(slot);
    }
    if (!has_victim) continue;
    if (!contains(victim) || !cooling_[slot_of_[victim]]) continue;  // rescued meanwhile: no eviction
    const uint32_t vslot = slot_of_[victim];
    berase(static_cast<uint32_t>(murmur64(victim) % B_), victim);
    slot_of_[victim] = kInv;
    cooling_[vslot] = 0;
    ++evicted;
    return vslot;
  }
}

void RecordCache::insert(uint32_t key, uint32_t dev, std::vector<CacheUpdate>& updates) {  // cache.hh:147-203
  const uint32_t slot = next_idx_ < C_ ? next_idx_++ : evict();
  updates.push_back({slot, dev, dev_of_[slot]});
  bpush(static_cast<uint32_t>(murmur64(key) % B_), key);
  slot_of_[key] = slot;
  key_of_[slot] = key;
  dev_of_[slot] = dev;
  cooling_[slot] = 0;
  ++admitted;
}

// (query, key) order of the candidates: an LSD radix sort over the composite (query << 32 | key), 16-bit digits, only
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
  std::vector<uint32_t> cnt(1u << 16);
  for (int shift = 0; shift < 64 && (most >> shift) != 0; shift += 16) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    for (size_t i = 0; i < n; ++i) ++cnt[(k[i] >> shift) & 0xFFFF];
    uint32_t sum = 0;
    for (uint32_t& x : cnt) {
      const uint32_t t = x;
      x = sum;
      sum += t;
    }
    for (size_t i = 0; i < n; ++i) {
      const uint32_t pos = cnt[(k[i] >> shift) & 0xFFFF]++;
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
                             std::vector<CacheUpdate>& updates, std::vector<uint32_t>& cool_on) {
  if (C_ == 0) return;
  cool_on_ = &cool_on;
  std::sort(rescued_keys.begin(), rescued_keys.end());
  rescued_keys.erase(std::unique(rescued_keys.begin(), rescued_keys.end()), rescued_keys.end());
  for (uint32_t key : rescued_keys) {  // cache.hh:128-132
    if (contains(key) && cooling_[slot_of_[key]] && ct_remove(key)) {
      cooling_[slot_of_[key]] = 0;
      ++rescued;
    }
  }
  sort_candidates(candidates);  // (query, key): a query offers a key once, so the order is total
  for (const CacheCandidate& c : candidates) {
    if (c.key >= slot_of_.size() || contains(c.key)) continue;  // admitted by an earlier miss (cache.hh:171-179)
    if (c.always || !full() || c.coin) insert(c.key, c.dev_id, updates);
  }
  cool_on_ = nullptr;
}

std::vector<uint32_t> RecordCache::keys() const {
  std::vector<uint32_t> out;
  for (uint32_t k : key_of_)
    if (k != kInv && contains(k) && key_of_[slot_of_[k]] == k) out.push_back(k);
  std::sort(out.begin(), out.end());
  return out;
}

}  // namespace shine
