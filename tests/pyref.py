"""A second, independent restatement of the reference query path in pure Python — test infrastructure.

It reads the dump bytes directly (src/node/node.hh:10-19, src/memory_node.hh:15-27), restates libstdc++'s
std::push_heap / std::pop_heap (bits/stl_heap.h: __push_heap, __adjust_heap, __pop_heap) instead of calling
them, and follows HNSW::knn / search_for_one / search_level (src/hnsw/hnsw.hh:253-476).  Used only for small,
integer-valued cases, where every f32 partial sum of a squared-L2 distance is exact and the order of the sums
is irrelevant, so agreement with oracle/oracle.cc is a check of the oracle's heap and control flow.
"""
from __future__ import annotations

import struct

import numpy as np


def _max_cmp(a, b):  # heap.hh:15-17
    return a[1] < b[1]


def _min_cmp(a, b):  # heap.hh:19-21
    return a[1] > b[1]


def push_heap(h, comp):  # std::push_heap: __push_heap(first, len-1, 0, value)
    value = h[-1]
    hole = len(h) - 1
    parent = (hole - 1) // 2
    while hole > 0 and comp(h[parent], value):
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = value


def pop_heap(h, comp):  # std::pop_heap then pop_back
    if len(h) > 1:
        n = len(h) - 1
        value = h[n]
        h[n] = h[0]
        hole, second = 0, 0
        while second < (n - 1) // 2:  # __adjust_heap
            second = 2 * (second + 1)
            if comp(h[second], h[second - 1]):
                second -= 1
            h[hole] = h[second]
            hole = second
        if (n & 1) == 0 and second == (n - 2) // 2:
            second = 2 * (second + 1)
            h[hole] = h[second - 1]
            hole = second - 1
        parent = (hole - 1) // 2  # __push_heap(first, hole, 0, value)
        while hole > 0 and comp(h[parent], value):
            h[hole] = h[parent]
            hole = parent
            parent = (hole - 1) // 2
        h[hole] = value
    h.pop()


class PyRef:
    def __init__(self, dumps, dim, M):
        self.shards = [bytes(np.asarray(d, dtype=np.uint8)) for d in dumps]
        self.dim, self.M = dim, M
        self.nl0 = 4 + 8 * 2 * M
        self.nlu = 4 + 8 * M

    def _rec(self, rp):
        return self.shards[rp >> 48], rp & ((1 << 48) - 1)

    def uid(self, rp):
        b, o = self._rec(rp)
        return struct.unpack_from("<I", b, o + 8)[0]

    def level(self, rp):
        b, o = self._rec(rp)
        return struct.unpack_from("<I", b, o + 12)[0]

    def comps(self, rp):
        b, o = self._rec(rp)
        return np.frombuffer(b, dtype=np.float32, count=self.dim, offset=o + 16)

    def neighbours(self, rp, lvl):  # node.cc:18-27 + neighborlist.hh:27-38
        b, o = self._rec(rp)
        off = o + 16 + 4 * self.dim + (0 if lvl == 0 else self.nl0 + (lvl - 1) * self.nlu)
        cnt = struct.unpack_from("<I", b, off)[0]
        return list(struct.unpack_from(f"<{cnt}Q", b, off + 4))

    def dist(self, q, rp):  # squared L2 — exact for integer-valued data
        d = q.astype(np.int64) - self.comps(rp).astype(np.int64)
        return float(np.float32(int((d * d).sum())))

    def knn(self, q, k, ef):
        st = dict(distcomps=0, visited_upper=0, visited_l0=0, lists_upper=0, lists_l0=0)
        ep = struct.unpack_from("<Q", self.shards[0], 8)[0]  # rdma_reads.hh:74-99
        st["visited_upper" if self.level(ep) > 0 else "visited_l0"] += 1
        closest = self.dist(q, ep)
        st["distcomps"] += 1
        nn = ep
        for lvl in range(self.level(ep), 0, -1):  # search_for_one (hnsw.hh:331-393)
            changed = True
            while changed:
                changed = False
                st["lists_upper"] += 1
                best = None
                for r in self.neighbours(nn, lvl):
                    st["visited_upper"] += 1
                    d = self.dist(q, r)
                    st["distcomps"] += 1
                    if d < closest:
                        closest, best, changed = d, r, True
                nn = best if changed else nn
        top = [(nn, self.dist(q, nn))]
        st["distcomps"] += 1
        nxt = [top[0]]  # search_level (hnsw.hh:406-476)
        visited = {nn}
        while nxt:
            c = nxt[0]
            pop_heap(nxt, _min_cmp)
            if c[1] > top[0][1]:
                break
            st["lists_l0"] += 1
            for r in self.neighbours(c[0], 0):
                if r in visited:
                    continue
                st["visited_l0"] += 1
                visited.add(r)
                far = top[0][1]
                d = self.dist(q, r)
                st["distcomps"] += 1
                if d < far or len(top) < ef:
                    nxt.append((r, d))
                    push_heap(nxt, _min_cmp)
                    if len(top) < ef:  # push_k (heap.hh:34-41)
                        top.append((r, d))
                        push_heap(top, _max_cmp)
                    elif d < top[0][1]:
                        pop_heap(top, _max_cmp)
                        top.append((r, d))
                        push_heap(top, _max_cmp)
        while len(top) > k:
            pop_heap(top, _max_cmp)
        return [self.uid(r) for r, _ in top], [d for _, d in top], st
