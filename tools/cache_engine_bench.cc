// Host timing of the dynamic cache's policy engine (csrc/cache.{h,cc}) at the skew grid's steady state, without a GPU:
// per slot a RecordCache of the cfg5-shaped 10M index at ratio 5 % (~660K entries, keys below 10M), filled, then calls
// of ~4K admission candidates (Zipf-skewed keys, coin passed) and ~4K rescued keys, one thread per slot as capi.cc's
// replay_all runs them.  Prints the policy's mean ms per slot-call and a digest of the final contents (for comparing
// engine builds: the digest must not change).
//
// Build: g++ -O3 -std=c++20 -march=x86-64-v3 -pthread -I../dm-hnsw-reference_amd/csrc cache_engine_bench.cc
//        ../dm-hnsw-reference_amd/csrc/cache.cc -o /tmp/cache_engine_bench
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "cache.h"

using namespace shine;

int main(int argc, char** argv) {
  const uint32_t entries = argc > 1 ? std::atoi(argv[1]) : 660000;
  const uint32_t key_space = argc > 2 ? std::atoi(argv[2]) : 10000000;
  const int slots = argc > 3 ? std::atoi(argv[3]) : 8;
  const int calls = argc > 4 ? std::atoi(argv[4]) : 40;
  const uint32_t per_call = 4000;
  std::vector<double> ms(slots, 0);
  std::vector<uint64_t> digest(slots, 0);
  std::vector<std::thread> th;
  for (int s = 0; s < slots; ++s)
    th.emplace_back([&, s] {
      RecordCache c(entries, 1234 + s, key_space);
      std::mt19937_64 rng(99 + s);
      // Zipf-ish keys: floor(key_space * u^3) concentrates on small keys, scattered by a multiplicative hash
      auto key = [&] {
        const double u = std::uniform_real_distribution<double>(0, 1)(rng);
        const uint64_t r = static_cast<uint64_t>(key_space * u * u * u);
        return static_cast<uint32_t>((r * 2654435761ull) % key_space);
      };
      std::vector<uint32_t> recent;
      double total = 0;
      int timed = 0;
      auto one = [&](uint32_t n, bool time_it) {
        std::vector<CacheCandidate> cand;
        for (uint32_t i = 0; i < n; ++i) {
          const uint32_t k = key();
          cand.push_back({i / 4, k, k, (rng() & 63) == 0, true});
        }
        std::vector<uint32_t> resc;
        for (uint32_t i = 0; i < per_call && !recent.empty(); ++i) resc.push_back(recent[rng() % recent.size()]);
        std::vector<CacheUpdate> ups;
        std::vector<uint32_t> cool_on;
        const auto t0 = std::chrono::steady_clock::now();
        c.apply_call(resc, cand, ups, cool_on);
        const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        recent.clear();  // the keys cooling now (canonical order, so engine builds draw the same rescues)
        for (uint32_t sl : cool_on)
          if (c.cooling(sl)) recent.push_back(c.slot_key(sl));
        std::sort(recent.begin(), recent.end());
        recent.erase(std::unique(recent.begin(), recent.end()), recent.end());
        if (time_it) {
          total += t;
          ++timed;
        }
        for (const auto& u : ups) digest[s] = digest[s] * 1000003ull + u.slot * 31ull + u.new_dev + (u.old_dev & 0xFF);
      };
      while (!c.full()) one(40000, false);
      for (int call = 0; call < 100; ++call) one(per_call, false);
      for (int call = 0; call < calls; ++call) one(per_call, true);
      ms[s] = timed ? total / timed : 0;
      digest[s] ^= c.admitted * 7 + c.evicted * 13 + c.rescued * 17;
    });
  for (auto& t : th) t.join();
  double sum = 0;
  uint64_t dg = 0;
  for (int s = 0; s < slots; ++s) {
    sum += ms[s];
    dg = dg * 31 + digest[s];
  }
  std::printf("policy %.3f ms per slot-call (mean of %d slots), digest %016llx\n", sum / slots, slots,
              static_cast<unsigned long long>(dg));
  return 0;
}
