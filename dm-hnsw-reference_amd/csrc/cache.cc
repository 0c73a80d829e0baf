// Dynamic record cache engine: cache::Cache + CoolingTable (src/cache/cache.hh:24-311, cooling_table.hh:52-98) at
// call granularity.  See cache.h.
#include "cache.h"

#include <sys/mman.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <new>

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
  mod60_ = FastMod(60);
  for (uint32_t i = 0; i < kAhead; ++i) push_draw(i);
  std::fill(key_of_.data(), key_of_.data() + entries, kInv);
  std::fill(dev_of_.data(), dev_of_.data() + entries, kInv);
}

bool RecordCache::size_ok(uint32_t entries) {
  const uint32_t ct = std::max<uint32_t>(
      1, static_cast<uint32_t>(std::ceil(entries / static_cast<double>(kCoolingBucketEntries) * kCoolingRatio)));
  return entries > kCoolingBucketEntries * ct;
}

uint64_t RecordCache::next_draw() {
  state_ += 0x9E3779B97F4A7C15ull;
  uint64_t z = state_;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void RecordCache::push_draw(uint32_t slot) {
  Draw& d = ring_[slot];
  d.v = next_draw();
  d.b = static_cast<uint32_t>(modB_(d.v));
  d.r60 = static_cast<uint32_t>(mod60_(d.v));
  if (C_) __builtin_prefetch(brec(d.b));
}

RecordCache::Draw RecordCache::rand() {
  const Draw d = ring_[head_];
  push_draw(head_);
  head_ = head_ + 1 == kAhead ? 0u : head_ + 1;
  return d;
}

namespace {
struct Pick60 {
  uint8_t t[60][6];
  constexpr Pick60() : t() {
    for (int r = 0; r < 60; ++r)
      for (int n = 1; n < 6; ++n) t[r][n] = static_cast<uint8_t>(r % n);
  }
};
constexpr Pick60 kPick60Table{};
}  // namespace

const uint8_t (&RecordCache::kPick60)[60][RecordCache::kInPlace + 1] = kPick60Table.t;

uint32_t RecordCache::bucket_of(uint32_t key) const { return static_cast<uint32_t>(modB_(murmur64(key))); }
uint32_t RecordCache::cool_of(uint32_t key) const { return static_cast<uint32_t>(modCT_(splitmix(key))); }

int RecordCache::bfind(uint32_t b, uint32_t key, Ent& e) const {
  const uint32_t* r = brec(b);
  const uint32_t n = bcount(r), in = n < kInPlace ? n : kInPlace;
  for (uint32_t i = 0; i < in; ++i)
    if (r[1 + 3 * i] == key) {
      e = {key, r[2 + 3 * i], r[3 + 3 * i], ((r[0] >> (16 + i)) & 1u) != 0};
      return static_cast<int>(i);
    }
  if (n > kInPlace) {
    const std::vector<uint32_t>& o = bover_.at(b);
    for (size_t i = 0; i < o.size(); i += 4)
      if (o[i] == key) {
        e = {key, o[i + 1], o[i + 2], o[i + 3] != 0};
        return static_cast<int>(kInPlace + i / 4);
      }
  }
  return -1;
}

uint32_t RecordCache::slot_of(uint32_t key) const {
  if (C_ == 0 || key >= key_space_) return kInv;
  Ent e;
  return bfind(bucket_of(key), key, e) >= 0 ? e.slot : kInv;
}

RecordCache::Ent RecordCache::bget(uint32_t b, uint32_t i) const {
  const uint32_t* r = brec(b);
  if (i < kInPlace) return {r[1 + 3 * i], r[2 + 3 * i], r[3 + 3 * i], ((r[0] >> (16 + i)) & 1u) != 0};
  const uint32_t* o = bover_.at(b).data() + 4 * (i - kInPlace);
  return {o[0], o[1], o[2], o[3] != 0};
}

void RecordCache::bset_cool(uint32_t b, uint32_t i, bool cool) {
  if (i < kInPlace) {
    uint32_t* r = brec(b);
    r[0] = cool ? r[0] | (1u << (16 + i)) : r[0] & ~(1u << (16 + i));
  } else {
    bover_[b][4 * (i - kInPlace) + 3] = cool ? 1u : 0u;
  }
}

void RecordCache::bpush(uint32_t b, uint32_t key, uint32_t slot, uint32_t dev) {
  uint32_t* r = brec(b);
  const uint32_t n = bcount(r);
  if (n < kInPlace) {
    r[1 + 3 * n] = key;
    r[2 + 3 * n] = slot;
    r[3 + 3 * n] = dev;
    r[0] &= ~(1u << (16 + n));
  } else {
    auto& o = bover_[b];
    o.insert(o.end(), {key, slot, dev, 0u});
  }
  ++r[0];
}

void RecordCache::berase(uint32_t b, uint32_t i) {
  uint32_t* r = brec(b);
  const uint32_t n = bcount(r), in = n < kInPlace ? n : kInPlace;
  if (i < in) {
    for (uint32_t j = i; j + 1 < in; ++j) {
      r[1 + 3 * j] = r[4 + 3 * j];
      r[2 + 3 * j] = r[5 + 3 * j];
      r[3 + 3 * j] = r[6 + 3 * j];
    }
    const uint32_t bits = r[0] >> 16, low = bits & ((1u << i) - 1u), high = (bits >> (i + 1)) << i;
    uint32_t nb = low | high;
    if (n > kInPlace) {  // the first entry past the in-place ones moves in
      auto it = bover_.find(b);
      const uint32_t* o = it->second.data();
      r[1 + 3 * (kInPlace - 1)] = o[0];
      r[2 + 3 * (kInPlace - 1)] = o[1];
      r[3 + 3 * (kInPlace - 1)] = o[2];
      nb = (nb & ~(1u << (kInPlace - 1))) | ((o[3] != 0 ? 1u : 0u) << (kInPlace - 1));
      it->second.erase(it->second.begin(), it->second.begin() + 4);
      if (it->second.empty()) bover_.erase(it);
    }
    r[0] = (n - 1) | ((nb & ((1u << kInPlace) - 1u)) << 16);
  } else {
    auto it = bover_.find(b);
    const size_t k = 4 * (i - kInPlace);
    it->second.erase(it->second.begin() + k, it->second.begin() + k + 4);
    if (it->second.empty()) bover_.erase(it);
    r[0] = (r[0] & 0xFFFF0000u) | (n - 1);
  }
}

bool RecordCache::ct_remove(uint32_t key) {  // cooling_table.hh:52-75
  uint32_t* r = &ct_[static_cast<size_t>(cool_of(key)) * kCW];
  uint32_t i = 0;
  while (i < r[0] && r[1 + i] != key) ++i;
  if (i == r[0]) return false;
  for (uint32_t j = i; j + 1 < r[0]; ++j) {
    r[1 + j] = r[2 + j];
    r[kCB + j] = r[kCB + 1 + j];
  }
  --r[0];
  return true;
}

bool RecordCache::ct_insert(uint32_t key, uint32_t b, uint32_t c, uint32_t& victim, uint32_t& vbucket) {
  uint32_t* r = &ct_[static_cast<size_t>(c) * kCW];  // cooling_table.hh:81-98
  bool pushed = false;
  if (r[0] == kCoolingBucketEntries) {  // the oldest (last) key leaves
    victim = r[kCoolingBucketEntries];
    vbucket = r[kCB + kCoolingBucketEntries - 1];
    --r[0];
    pushed = true;
  }
  for (uint32_t j = r[0]; j > 0; --j) {  // newest first
    r[1 + j] = r[j];
    r[kCB + j] = r[kCB + j - 1];
  }
  r[1] = key;
  r[kCB] = b;
  ++r[0];
  return pushed;
}

// The draw i ahead of the stream without taking it (1 <= i <= kAhead; prefetch hints only).
const RecordCache::Draw& RecordCache::peek(uint32_t i) const { return ring_[(head_ + i - 1) % kAhead]; }

// The next pick of the eviction scan, read ahead (its bucket's line was requested kAhead draws earlier): when the
// step will start an entry cooling, its cooling-table bucket is computed now (kept for that step: cool_bucket) and —
// when that bucket is full — the hash record of the key it would push out is requested, so that the victim lookup,
// the scan's one dependent miss, overlaps this step's.  A hint only: the step itself re-reads everything.
void RecordCache::lookahead() {
  const Draw& d1 = peek(1);
  const uint32_t* r = brec(d1.b);
  const uint32_t n = bcount(r);
  if (n == 0 || n > kInPlace) return;
  const uint32_t i = pick(peek(2), n);
  if ((r[0] >> (16 + i)) & 1u) return;  // already cooling: the step changes nothing
  memo_key_ = r[1 + 3 * i];
  memo_cool_ = cool_of(memo_key_);
  const uint32_t* c = &ct_[static_cast<size_t>(memo_cool_) * kCW];
  if (c[0] == kCoolingBucketEntries) __builtin_prefetch(brec(c[kCB + kCoolingBucketEntries - 1]));
}

RecordCache::Victim RecordCache::evict() {  // cache.hh:232-311
  for (;;) {
    ++scan_steps;
    const uint32_t b = rand().b;  // (its record was requested kAhead draws ago)
    const uint32_t n = bcount(brec(b));
    if (n == 0) continue;
    const uint32_t i = pick(rand(), n);
    const Ent e = bget(b, i);
    const uint32_t cb = e.cool ? 0u : cool_bucket(e.key);  // (before the look-ahead overwrites its memo)
    lookahead();
    uint32_t victim = kInv, vb = 0;
    bool has_victim = false;
    if (!e.cool) {  // hot -> cooling; the table may push its oldest key out
      has_victim = ct_insert(e.key, b, cb, victim, vb);
      bset_cool(b, i, true);
      cooling_[e.slot] = 1;
      if (flagged_) flagged_->push_back(e.slot);
    }
    if (!has_victim) continue;
    Ent v;
    const int vi = bfind(vb, victim, v);
    if (vi < 0 || !v.cool) continue;  // rescued meanwhile: no eviction
    berase(vb, static_cast<uint32_t>(vi));
    cooling_[v.slot] = 0;
    ++evicted;
    return {v.slot, v.dev};
  }
}

void RecordCache::insert(uint32_t key, uint32_t dev, std::vector<CacheUpdate>& updates) {  // cache.hh:147-203
  const Victim v = next_idx_ < C_ ? Victim{next_idx_++, kInv} : evict();
  updates.push_back({v.slot, dev, v.dev});
  bpush(bucket_of(key), key, v.slot, dev);
  key_of_[v.slot] = key;
  dev_of_[v.slot] = dev;
  cooling_[v.slot] = 0;
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
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const clk::time_point t0 = clk::now();
  scan_steps = 0;
  flagged_ = &flagged;
  if (!std::is_sorted(rescued_keys.begin(), rescued_keys.end())) std::sort(rescued_keys.begin(), rescued_keys.end());
  rescued_keys.erase(std::unique(rescued_keys.begin(), rescued_keys.end()), rescued_keys.end());
  constexpr size_t kLookAhead = 8;  // lookups requested this many keys ahead (each one a likely miss)
  const size_t nr = rescued_keys.size();
  for (size_t i = 0; i < nr; ++i) {  // cache.hh:128-132
    if (i + kLookAhead < nr && rescued_keys[i + kLookAhead] < key_space_) {
      const uint32_t k = rescued_keys[i + kLookAhead];
      __builtin_prefetch(brec(bucket_of(k)));
      __builtin_prefetch(&ct_[static_cast<size_t>(cool_of(k)) * kCW]);
    }
    const uint32_t key = rescued_keys[i];
    if (key >= key_space_) continue;
    const uint32_t b = bucket_of(key);
    Ent e;
    const int at = bfind(b, key, e);
    if (at >= 0 && e.cool && ct_remove(key)) {
      bset_cool(b, static_cast<uint32_t>(at), false);
      cooling_[e.slot] = 0;
      flagged.push_back(e.slot);
      ++rescued;
    }
  }
  const clk::time_point t1 = clk::now();
  sort_candidates(candidates);  // (query, key): a query offers a key once, so the order is total
  const clk::time_point t2 = clk::now();
  const size_t nc = candidates.size();
  for (size_t i = 0; i < nc; ++i) {
    if (i + kLookAhead < nc && candidates[i + kLookAhead].key < key_space_)
      __builtin_prefetch(brec(bucket_of(candidates[i + kLookAhead].key)));
    const CacheCandidate& c = candidates[i];
    if (c.key >= key_space_ || contains(c.key)) continue;  // admitted by an earlier miss (cache.hh:171-179)
    if (c.always || !full() || c.coin) insert(c.key, c.dev_id, updates);
  }
  flagged_ = nullptr;
  const clk::time_point t3 = clk::now();
  ms_rescue = ms(t0, t1);
  ms_sort = ms(t1, t2);
  ms_admit = ms(t2, t3);
}

std::vector<uint32_t> RecordCache::keys() const {
  std::vector<uint32_t> out;
  for (size_t s = 0; s < key_of_.size(); ++s)
    if (const uint32_t k = key_of_[s]; k != kInv && slot_of(k) == s) out.push_back(k);
  std::sort(out.begin(), out.end());
  return out;
}

}  // namespace shine
