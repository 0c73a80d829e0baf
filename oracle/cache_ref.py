"""Restatement of the compute node's record cache (cache::Cache + CoolingTable) at batch granularity — TEST
INFRASTRUCTURE ONLY (the checker for SHINE_CACHE_DYNAMIC).  Only tests/ may import this module.

The reference cache (src/cache/cache.hh:24-311, cooling_table.hh:52-98) admits node records on a miss (hnsw.hh:524-548:
upper-level nodes always (:368), level-0 nodes while the cache is not full and then with probability ADMISSION_RATIO
= 0.01 (:447-448, constants.hh:16)), evicts through random cooling (cache.hh:232-311: pick a random bucket and a
random entry in it; an entry that is not cooling enters the cooling table's FIFO bucket, which pushes its oldest
key out; that key is evicted if it is still cooling) and gives a cooling entry a second chance when it is hit
(cache.hh:128-132: removed from the cooling table, no longer cooling).  Capacity: cache_size / (16 + 4d) entries with
cache_size = ratio % of estimate_index_size (compute_node.cc:40-56, hnsw.hh:309-321); as many hash buckets as entries;
ceil(entries / 6 * 0.1) cooling buckets of 6 (constants.hh:14-15).

The GPU engine applies this policy between calls (capi.cc DynCache): during a call the cache is fixed; every record
read of a query is a hit (its key is cached) or a miss; after the call the hit cooling entries are rescued (keys in
ascending order), then the misses are offered for admission in (query, key) order — a key already admitted by an
earlier miss is a no-op, as a concurrent insert of a present key is in cache.hh:171-179 — admitted when
always-admitted (entry point, upper levels), or the cache is not full at that moment, or its coin passed (a hash of
(seed, call, query, device id) below 0.01).  The reference draws its randomness from an unseeded std::random_device;
here one SplitMix64 stream per cache (seeded) drives the eviction draws, and keys are record uids (the RemotePtr of
the reference names the same record).  This module is the same policy written independently, so a GPU run and this
restatement must agree on every hit count and on the cache contents after every call.
"""
from __future__ import annotations

import math

MASK = (1 << 64) - 1
ADMISSION_RATIO = 0.01          # constants.hh:16
COOLING_TABLE_BUCKET_ENTRIES = 6  # constants.hh:14
COOLING_TABLE_RATIO = 0.1       # constants.hh:15


def murmur64(x: int) -> int:  # std::hash<RemotePtr> (remote_pointer.hh:31-51) over the key
    x &= MASK
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & MASK
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & MASK
    x ^= x >> 33
    return x


def splitmix_fmix(z: int) -> int:  # cooling_table.hh hash (SplitMix64 finaliser)
    z = (z + 0x9E3779B97F4A7C15) & MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def admission_coin(seed: int, call: int, query: int, dev_id: int) -> bool:
    """The coin a level-0 miss draws once the cache is full (hnsw.hh:447-448 admit_to_cache(ADMISSION_RATIO))."""
    z = (seed + 0x9E3779B97F4A7C15 * (call + 1) + 0xC2B2AE3D27D4EB4F * (query + 1) + 0x165667B19E3779F9 * (dev_id + 1)) & MASK
    h = splitmix_fmix(z)
    return (h >> 40) < int(ADMISSION_RATIO * (1 << 24))


def _round(x: float) -> int:  # std::round: halves away from zero (Python's round() goes to even)
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def estimate_index_size(n: int, M: int, dim: int) -> int:  # hnsw.hh:309-321, node.hh:44-54
    levels = _round(math.log(n) / math.log(M))
    size = 0
    for i in range(levels):
        s = (16 + 4 * dim) + (4 + 8 * 2 * M) if i == 0 else 4 + 8 * M
        size += _round((1.0 / M) ** i * n) * s
    return size


def capacity(n: int, M: int, dim: int, ratio_percent: float) -> int:  # compute_node.cc:40-54
    import numpy as np
    cache_size = int(float(np.float32(estimate_index_size(n, M, dim))) / 100.0 * ratio_percent)
    return cache_size // (16 + 4 * dim)


class RefCache:
    def __init__(self, entries: int, seed: int):
        self.C = entries
        self.B = max(1, entries)
        self.CT = max(1, math.ceil(entries / COOLING_TABLE_BUCKET_ENTRIES * COOLING_TABLE_RATIO))
        self.buckets = [[] for _ in range(self.B)]  # keys, insertion order (cache.hh Bucket list)
        self.ct = [[] for _ in range(self.CT)]      # newest first (cooling_table.hh:81-98)
        self.cooling = {}                           # key -> bool, for every cached key
        self.next_idx = 0
        self.state = seed & MASK
        self.admitted = self.evicted = self.rescued = 0

    def rand(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
        return z ^ (z >> 31)

    def __contains__(self, key) -> bool:
        return key in self.cooling

    def is_full(self) -> bool:  # cache.hh:205-216
        return self.next_idx >= self.C

    def ct_insert(self, key):  # cooling_table.hh:81-98
        b = self.ct[splitmix_fmix(key) % self.CT]
        victim = b.pop() if len(b) == COOLING_TABLE_BUCKET_ENTRIES else None
        b.insert(0, key)
        return victim

    def ct_remove(self, key) -> bool:  # cooling_table.hh:52-75
        b = self.ct[splitmix_fmix(key) % self.CT]
        if key in b:
            b.remove(key)
            return True
        return False

    def rescue(self, key):  # cache.hh:128-132: a hit on a cooling entry
        if self.cooling.get(key) and self.ct_remove(key):
            self.cooling[key] = False
            self.rescued += 1

    def evict(self):  # cache.hh:232-311; returns the evicted key
        while True:
            b = self.buckets[self.rand() % self.B]
            if not b:
                continue
            key = b[self.rand() % len(b)]
            victim = None
            if not self.cooling[key]:
                victim = self.ct_insert(key)
                self.cooling[key] = True
            if victim is not None and self.cooling.get(victim):
                self.buckets[murmur64(victim) % self.B].remove(victim)
                del self.cooling[victim]
                self.evicted += 1
                return victim

    def insert(self, key):  # cache.hh:147-203 (no concurrent duplicate: keys are offered once)
        if self.next_idx < self.C:
            self.next_idx += 1
        else:
            self.evict()
        self.buckets[murmur64(key) % self.B].append(key)
        self.cooling[key] = False
        self.admitted += 1

    def apply_call(self, rescued_keys, candidates):
        """After a call: rescues (ascending keys), then candidates [(query, key, always, coin)] in (query, key) order,
        a key not yet cached admitted if always, or not full now, or its coin passed."""
        for key in sorted(set(rescued_keys)):
            self.rescue(key)
        for q, key, always, coin in sorted(candidates, key=lambda c: (c[0], c[1])):
            if key in self:  # admitted by an earlier miss of this call
                continue
            if always or not self.is_full() or coin:
                self.insert(key)

    def keys(self):
        return set(self.cooling)
