// Stress test of shine::TaskPool (csrc/index_internal.h), the handle's worker pool for the dynamic cache's per-slot
// replays: 20,000 runs of 1-9 tasks, the pool growing while it is in use; every task must run exactly once per run.
// Built and run by tests/test_task_pool.py under ThreadSanitizer (host code only).
#include "index_internal.h"
#include <cstdio>
#include <atomic>
int main() {
  shine::TaskPool pool;
  std::atomic<long> total{0};
  for (int rep = 0; rep < 20000; ++rep) {
    const size_t n = 1 + rep % 9;
    std::vector<int> hit(n, 0);
    pool.run(n, [&](size_t i) { hit[i]++; total += i; });
    for (size_t i = 0; i < n; ++i) if (hit[i] != 1) { std::printf("FAIL rep %d i %zu hit %d\n", rep, i, hit[i]); return 1; }
  }
  std::printf("pool ok %ld\n", total.load());
}
