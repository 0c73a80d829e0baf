"""CPU restatement of the reference's region placement and query routing — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; it is the checker for csrc/placement.cc (shine_kmeans, shine_router_run,
shine_plan_regions), never part of the product path.  It restates, in numpy float32 arithmetic:
  * Kmeans<Distance>: init_plusplus (src/cache/kmeans.hh:163-197), compute_cluster_assignment (202-223),
    calculate_means (225-252), run_kmeans (93-137), balanced_kmeans (259-377), run_and_optimize (24-91);
  * Placement::closest_centroids (src/cache/placement.hh:63-72): a MinPlacement heap of (mapping[i], distance),
    popped in libstdc++'s std::push_heap / std::pop_heap order;
  * QueryRouter::update_limits (src/router/query_router.hh:106-151) and the routing loop of run_routing (280-387)
    with BALANCED_ROUTING / ADAPTIVE_ROUTING and LIMIT_PER_CN = 200 (src/common/constants.hh:20-25).
std::mt19937{1234} is Python's MT19937 with init_genrand state; std::uniform_int_distribution<size_t> is libstdc++'s
Lemire downscaling (bits/uniform_int_dist.h, GCC 11).  Distances follow hostdist.h's order (8 lane FMA accumulators,
left-to-right lane sum, scalar tail); each FMA is evaluated in float64 and rounded once to float32, which is exact
for the integer-valued inputs the tests use (every product and partial sum then fits 53 bits).
Small cases only: pure-Python loops.
"""
from __future__ import annotations

import random

import numpy as np

F32 = np.float32
FLT_MAX = F32(np.finfo(np.float32).max)
ITERATION_LIMIT = 1000  # kmeans.hh:12
LIMIT_PER_CN = 200      # constants.hh:25


# ---- std::mt19937 / std::uniform_int_distribution<size_t> ----------------------------------------------------------
def mt19937(seed: int) -> random.Random:
    mt = random.Random()
    mt.seed(0)
    st = list(mt.getstate())
    key = [seed & 0xFFFFFFFF]
    for i in range(1, 624):  # init_genrand
        key.append((1812433253 * (key[-1] ^ (key[-1] >> 30)) + i) & 0xFFFFFFFF)
    mt.setstate((st[0], tuple(key + [624]), st[2]))
    return mt


def uniform_index(mt: random.Random, lo: int, hi: int) -> int:
    """uniform_int_distribution<size_t>(lo, hi) over a 32-bit engine: _S_nd<uint64_t>(urng, hi - lo + 1)."""
    rng = hi - lo + 1
    prod = mt.getrandbits(32) * rng
    low = prod & 0xFFFFFFFF
    if low < rng:
        threshold = ((1 << 32) - rng) % rng
        while low < threshold:
            prod = mt.getrandbits(32) * rng
            low = prod & 0xFFFFFFFF
    return lo + (prod >> 32)


# ---- distances (hostdist.h order) ----------------------------------------------------------------------------------
def _fma(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def dist_many(metric: int, X: np.ndarray, y: np.ndarray) -> np.ndarray:
    """Distance::dist(X[i], y) for every row: L2Distance (metric 0) or IPDistance = 1 - <x, y> (metric 1)."""
    X = np.asarray(X, np.float32).reshape(-1, np.asarray(y).shape[-1])
    y = np.asarray(y, np.float32)
    d = X.shape[1]
    q16 = d >> 4 << 4
    acc = np.zeros((X.shape[0], 8), np.float32)
    for i in range(0, q16, 8):
        if metric == 0:
            t = X[:, i:i + 8] - y[i:i + 8]
            acc = _fma(t, t, acc)
        else:
            acc = _fma(X[:, i:i + 8], np.broadcast_to(y[i:i + 8], (X.shape[0], 8)), acc)
    r = acc[:, 0].copy()
    for j in range(1, 8):
        r = r + acc[:, j]
    if metric == 0:
        for i in range(q16, d):
            t = X[:, i] - y[i]
            r = _fma(t, t, r)
        return r
    t = np.zeros(X.shape[0], np.float32)
    for i in range(q16, d):
        t = _fma(X[:, i], np.full(X.shape[0], y[i], np.float32), t)
    return F32(1.0) - (r + t)


def dist(metric: int, a: np.ndarray, b: np.ndarray) -> np.float32:
    return dist_many(metric, np.asarray(a, np.float32)[None, :], b)[0]


# ---- Kmeans --------------------------------------------------------------------------------------------------------
def init_plusplus(metric, rows, k):
    n = rows.shape[0]
    chosen = [uniform_index(mt19937(1234), 0, n - 1)]
    while len(chosen) < k:
        closest = np.full(n, FLT_MAX, np.float32)
        for j in chosen:  # closest_distances: strict < against every chosen centre, in order
            t = dist_many(metric, rows, rows[j])
            closest = np.where(t < closest, t, closest)
        chosen.append(int(np.argmax(closest)))  # std::max_element: the first maximum
    return rows[chosen].astype(np.float32).copy()


def assign(metric, rows, centroids):
    best = np.full(rows.shape[0], FLT_MAX, np.float32)
    idx = np.zeros(rows.shape[0], np.int64)
    for c in range(centroids.shape[0]):
        t = dist_many(metric, rows, centroids[c])
        better = t < best
        best = np.where(better, t, best)
        idx = np.where(better, c, idx)
    return idx


def calculate_means(rows, asg, old, k):
    c = np.zeros_like(old)
    count = np.zeros(k, np.float32)
    for i in range(rows.shape[0]):
        count[asg[i]] += F32(1)
        c[asg[i]] = c[asg[i]] + rows[i]
    for i in range(k):
        if count[i] == 0:
            c[i] = old[i]
        else:
            c[i] = c[i] / count[i]
    return c


def run_kmeans(metric, rows, k):
    rows = np.asarray(rows, np.float32)
    error = FLT_MAX
    it = 0
    centroids = asg = None
    while it < ITERATION_LIMIT and float(error) > 0.001:
        nc = init_plusplus(metric, rows, k) if it == 0 else calculate_means(rows, asg, centroids, k)
        asg = assign(metric, rows, nc)
        if it > 0:
            error = F32(0)
            for i in range(k):
                t = dist(metric, centroids[i], nc[i])
                error = error + (np.sqrt(t) if metric == 0 else t)
        centroids = nc
        it += 1
    sizes = np.bincount(asg, minlength=k).astype(np.int64)
    return centroids, asg, sizes, it


def balanced_kmeans(metric, rows, k, centroids, asg, sizes, c=F32(0.15), penalty_factor=F32(1.01), max_diff=1):
    rows = np.asarray(rows, np.float32)
    centroids = centroids.copy()
    asg = asg.copy()
    sizes = [int(s) for s in sizes]
    n = rows.shape[0]
    p_now, p_next = F32(0), FLT_MAX
    n_min, n_max, it = 0, n, 0
    s = np.zeros_like(centroids)
    for i in range(n):
        s[asg[i]] = s[asg[i]] + rows[i]
    with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
        while n_max - n_min > max_diff and it < ITERATION_LIMIT:
            for ni in range(n):
                x = rows[ni]
                old = int(asg[ni])
                if sizes[old] == 1:
                    continue
                s[old] = s[old] - x
                centroids[old] = s[old] / F32(sizes[old] - 1)
                sizes[old] -= 1
                cost = FLT_MAX
                dist_old = dist(metric, centroids[old], x)
                old_size = F32(sizes[old]) + c
                dj = dist_many(metric, centroids, x)  # centroids change only after the scan
                dest = old
                for j in range(k):
                    dist_j = dj[j]
                    size_j = F32(sizes[j])
                    needed = (dist_j - dist_old) / (old_size - size_j)
                    if old_size > size_j:
                        if p_now < needed:
                            if needed < p_next:
                                p_next = needed
                        elif dist_j + p_now * size_j < cost and j != old:
                            cost = dist_j + p_now * size_j
                            dest = j
                    elif p_now < needed and dist_j + p_now * size_j < cost:
                        cost = dist_j + p_now * size_j
                        dest = j
                asg[ni] = dest
                s[dest] = s[dest] + x
                centroids[dest] = s[dest] / F32(sizes[dest] + 1)
                sizes[dest] += 1
            n_min, n_max = min(sizes), max(sizes)
            p_now = penalty_factor * p_next
            p_next = FLT_MAX
            it += 1
    actual = np.bincount(assign(metric, rows, centroids), minlength=k).astype(np.int64)
    return centroids, asg, actual, it


def run_and_optimize(metric, rows, k, balanced=True):
    """(centroids, mapping, region sizes, Lloyd iterations, balancing iterations)."""
    if not balanced:
        cent, _, sizes, it = run_kmeans(metric, rows, k)
        return cent, np.arange(k), sizes, it, 0
    local_k = k if k % 2 == 0 else 2 * k
    cent, asg, sizes, it = run_kmeans(metric, rows, local_k)
    cent, asg, bal, bit = balanced_kmeans(metric, rows, local_k, cent, asg, sizes)
    if k % 2 == 0:
        return cent, np.arange(k), bal, it, bit
    mapping = np.zeros(local_k, np.int64)
    out_sizes = np.zeros(k, np.int64)
    paired = [False] * local_k
    nxt = 0
    for i in range(local_k):
        if paired[i]:
            continue
        min_dist, min_pos = FLT_MAX, 0
        for j in range(i + 1, local_k):
            if not paired[j]:
                t = dist(metric, cent[i], cent[j])
                if t < min_dist:
                    min_dist, min_pos = t, j
        assert min_pos != i, "invalid assignment"
        paired[i] = paired[min_pos] = True
        mapping[i] = mapping[min_pos] = nxt
        out_sizes[nxt] = bal[i] + bal[min_pos]
        nxt += 1
    return cent, mapping, out_sizes, it, bit


# ---- Placement::closest_centroids ----------------------------------------------------------------------------------
def _cmp(a, b):  # MinHeapPlacementCompare: lhs.second > rhs.second
    return a[1] > b[1]


def _push_heap(h):
    value = h[-1]
    hole = len(h) - 1
    parent = (hole - 1) // 2
    while hole > 0 and _cmp(h[parent], value):
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = value


def _pop_heap(h):
    if len(h) > 1:
        n = len(h) - 1
        value = h[n]
        h[n] = h[0]
        hole = second = 0
        while second < (n - 1) // 2:
            second = 2 * (second + 1)
            if _cmp(h[second], h[second - 1]):
                second -= 1
            h[hole] = h[second]
            hole = second
        if (n & 1) == 0 and second == (n - 2) // 2:
            second = 2 * (second + 1)
            h[hole] = h[second - 1]
            hole = second - 1
        parent = (hole - 1) // 2
        while hole > 0 and _cmp(h[parent], value):
            h[hole] = h[parent]
            hole = parent
            parent = (hole - 1) // 2
        h[hole] = value
    h.pop()


def closest_regions(metric, centroids, mapping, x):
    d = dist_many(metric, centroids, x)
    h = []
    for i in range(centroids.shape[0]):
        h.append((int(mapping[i]), d[i]))
        _push_heap(h)
    order = []
    while h:
        order.append(h[0][0])
        _pop_heap(h)
    return order


# ---- QueryRouter ---------------------------------------------------------------------------------------------------
def update_limits(limits, progresses, k):
    total = float(sum(int(p) for p in progresses) & 0xFFFFFFFF)  # std::accumulate(..., 0u)
    if total < k or k < 2:
        return limits
    denom = 0.0
    for i in range(k):
        denom += total - progresses[i]
    new = []
    nb = 0
    for i in range(k):
        scale = ((total - progresses[i]) / denom) * float(k)
        new.append(int(float(LIMIT_PER_CN) * scale))
        nb += new[-1]
    i = 0
    while nb < LIMIT_PER_CN * k:
        new[i % k] += 1
        nb += 1
        i += 1
    return new


def route(metric, centroids, mapping, k, queries, queue_sizes=None, adaptive=True):
    """Region of every query and the final limits; queue_sizes[b] at boundary b (the last row repeats)."""
    batch = LIMIT_PER_CN * k
    limits = [LIMIT_PER_CN] * k
    hist = [0] * k
    out = []
    boundary = 0
    for slot in range(queries.shape[0]):
        if slot > 0 and slot % batch == 0:
            hist = [0] * k
            if adaptive:
                p = [0] * k
                if queue_sizes is not None and len(queue_sizes):
                    p = [int(v) for v in queue_sizes[min(boundary, len(queue_sizes) - 1)]]
                boundary += 1
                limits = update_limits(limits, p, k)
        dest = 0
        for c in closest_regions(metric, centroids, mapping, queries[slot]):
            dest = c
            if hist[dest] < limits[dest]:
                break
        hist[dest] += 1
        out.append(dest)
    return np.array(out, np.uint32), np.array(limits, np.uint64)
