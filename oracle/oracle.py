"""ctypes wrapper of liboracle.so — TEST INFRASTRUCTURE ONLY (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "liboracle.so"
# The same restatement built with the reference's flags (-O3 -march=native -ffast-math -mavx2, CMakeLists.txt:16)
# for the CPU baseline only: -march=native must target the host that times it, so bench.py builds it there
# (`make -C oracle native`).  Its distances may differ in the last bit (contraction / reassociation): never a checker.
NATIVE_PATH = ORACLE_DIR / "liboracle_native.so"
NATIVE_FLAGS = "-O3 -march=native -ffast-math -mavx2"
QS_WORDS = 8
_libs = {}


def lib(path: Path = LIB_PATH):
    if path not in _libs:
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(str(path))
        P, U32, I32 = C.c_void_p, C.c_uint32, C.c_int
        L.oracle_draw_levels.argtypes = [U32, U32, U32, U32, P, P]
        L.oracle_build.restype = P
        L.oracle_build.argtypes = [P, U32, U32, U32, U32, I32, U32, U32]
        L.oracle_dump_size.restype = C.c_uint64
        L.oracle_dump_size.argtypes = [P, U32]
        L.oracle_dump_data.restype = P
        L.oracle_dump_data.argtypes = [P, U32]
        L.oracle_build_distcomps.restype = C.c_uint64
        L.oracle_build_distcomps.argtypes = [P]
        L.oracle_max_level.restype = U32
        L.oracle_max_level.argtypes = [P]
        L.oracle_open.restype = P
        L.oracle_open.argtypes = [P, P, U32, U32, U32, I32]
        L.oracle_free.argtypes = [P]
        L.oracle_knn.restype = I32
        L.oracle_knn.argtypes = [P, P, U32, U32, U32, P, P, P, U32]
        L.oracle_knn_trace.restype = I32
        L.oracle_knn_trace.argtypes = [P, P, U32, U32, U32, P, P, P, P, P, C.c_uint64, P]
        L.oracle_knn_pinned.restype = I32
        L.oracle_knn_pinned.argtypes = [P, P, U32, U32, U32, P, P, P, U32, P]
        L.oracle_distance.restype = C.c_float
        L.oracle_distance.argtypes = [I32, P, P, U32]
        L.oracle_selftest_heap.restype = I32
        L.oracle_selftest_heap.argtypes = [I32, P, P, P, U32, U32, P, P, P]
        _libs[path] = L
    return _libs[path]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def draw_levels(n, M, seed, n_shards=1):
    lv = np.empty(n, np.uint32)
    sh = np.empty(n, np.uint32)
    lib().oracle_draw_levels(n, M, seed, n_shards, _p(lv), _p(sh))
    return lv, sh


def build(base: np.ndarray, M: int, efc: int, metric: int = 0, n_shards: int = 1, seed: int = 1234):
    """Single-threaded HNSW::insert in slot order.  Returns (dumps, build_distcomps, max_level)."""
    b = np.ascontiguousarray(base, dtype=np.float32)
    h = lib().oracle_build(_p(b), b.shape[0], b.shape[1], M, efc, metric, n_shards, seed)
    try:
        dumps = []
        for s in range(n_shards):
            n = lib().oracle_dump_size(h, s)
            p = lib().oracle_dump_data(h, s)
            dumps.append(np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n,)).copy())
        return dumps, int(lib().oracle_build_distcomps(h)), int(lib().oracle_max_level(h))
    finally:
        lib().oracle_free(h)


class OracleIndex:
    def __init__(self, dumps, dim, M, metric=0, native=False):
        """native=True: the reference-flags build (CPU baseline timing only)."""
        self._lib = lib(NATIVE_PATH if native else LIB_PATH)
        self._dumps = [np.ascontiguousarray(d, dtype=np.uint8) for d in dumps]
        ptrs = (C.c_void_p * len(dumps))(*[d.ctypes.data for d in self._dumps])
        sizes = (C.c_uint64 * len(dumps))(*[d.size for d in self._dumps])
        self._h = self._lib.oracle_open(ptrs, sizes, len(dumps), dim, M, metric)
        self.dim = dim

    def knn(self, queries, k, ef, threads=1, cpus=None):
        """cpus: pin worker t to CPU cpus[t] (len(cpus) == threads)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq = q.shape[0]
        ids = np.empty((nq, k), np.uint32)
        dd = np.empty((nq, k), np.float32)
        qs = np.empty((nq, QS_WORDS), np.uint32)
        if cpus is not None:
            cp = np.ascontiguousarray(cpus, np.int32)
            assert cp.size == threads
            rc = self._lib.oracle_knn_pinned(self._h, _p(q), nq, k, ef, _p(ids), _p(dd), _p(qs), threads, _p(cp))
        else:
            rc = self._lib.oracle_knn(self._h, _p(q), nq, k, ef, _p(ids), _p(dd), _p(qs), threads)
        if rc != 0:
            raise RuntimeError(f"oracle_knn failed: {rc}")
        return ids, dd, qs

    def knn_trace(self, queries, k, ef, cap_per_query=None):
        """knn (one thread) plus every query's record reads in order: (uids, always, memory_nodes, offsets); reads
        offsets[i]:offsets[i+1] belong to query i, always = entry point / upper-level node (admitted without the coin)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        nq = q.shape[0]
        cap = nq * (cap_per_query or 64 * ef + 1024)
        ids = np.empty((nq, k), np.uint32)
        dd = np.empty((nq, k), np.float32)
        qs = np.empty((nq, QS_WORDS), np.uint32)
        reads = np.empty(cap, np.uint32)
        nodes = np.empty(cap, np.uint16)
        off = np.zeros(nq + 1, np.uint64)
        rc = self._lib.oracle_knn_trace(self._h, _p(q), nq, k, ef, _p(ids), _p(dd), _p(qs), _p(reads), _p(nodes), cap,
                                        _p(off))
        if rc != 0:
            raise RuntimeError(f"oracle_knn_trace failed: {rc}")
        n = int(off[-1])
        return (ids, dd, qs), (reads[:n] >> 1, (reads[:n] & 1).astype(bool), nodes[:n].copy(), off.astype(np.int64))

    def close(self):
        if self._h:
            self._lib.oracle_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def distance(metric, a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return float(lib().oracle_distance(metric, _p(a), _p(b), a.shape[0]))


def heap_replay(is_max, ops, vals, ids, k=0):
    ops = np.ascontiguousarray(ops, np.int32)
    vals = np.ascontiguousarray(vals, np.float32)
    ids = np.ascontiguousarray(ids, np.uint32)
    od = np.empty(len(ops) + 1, np.float32)
    oi = np.empty(len(ops) + 1, np.uint32)
    on = np.zeros(1, np.uint32)
    lib().oracle_selftest_heap(int(is_max), _p(ops), _p(vals), _p(ids), len(ops), k, _p(od), _p(oi), _p(on))
    n = int(on[0])
    return od[:n].copy(), oi[:n].copy()
