"""Host-side API over the C ABI, shaped after the reference's query interface.

`Index` plays the memory-node tier plus `HNSW<Distance>` (src/memory_node.hh, src/hnsw/hnsw.hh): it is opened
from the memory nodes' dumps and answers `knn` for a batch.  `build()` runs the parallel restatement of
`HNSW::insert` and returns the dump images.  Device-pointer entry points take raw integers (e.g.
`tensor.data_ptr()`) so that torch stays plumbing.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _dump_arrays(dumps):
    dumps = [np.ascontiguousarray(np.frombuffer(d, dtype=np.uint8) if not isinstance(d, np.ndarray) else d,
                                  dtype=np.uint8) for d in dumps]
    ptrs = (C.POINTER(C.c_uint8) * len(dumps))(*[d.ctypes.data_as(C.POINTER(C.c_uint8)) for d in dumps])
    sizes = (C.c_uint64 * len(dumps))(*[d.size for d in dumps])
    return dumps, ptrs, sizes


def _gpus(gpus):
    if not gpus:
        return None, 0
    arr = (C.c_int * len(gpus))(*gpus)
    return arr, len(gpus)


def _placement(p) -> int:
    if isinstance(p, int):
        return p
    try:
        return {"replica": L.PLACE_REPLICA, "sharded": L.PLACE_SHARDED, "regions": L.PLACE_SHARDED_REGIONS}[p]
    except KeyError:
        raise ValueError(f"placement must be 'replica', 'sharded' or 'regions', not {p!r}") from None


@dataclass
class KnnResult:
    ids: np.ndarray      # (nq, k) uint32 uids, reference result order (heap-array order)
    dists: np.ndarray    # (nq, k) float32
    qstats: np.ndarray   # (nq, QS_WORDS) uint32, SHINE_QS_* layout
    stats: dict          # aggregates (statistics.hh names)


class KnnRequest:
    """A shine_knn_batch_async call in flight: its output arrays are filled by wait()."""

    def __init__(self, req: C.c_void_p, res: KnnResult):
        self._req = req
        self._res = res

    def wait(self) -> KnnResult:
        if self._req is None:
            return self._res
        st = L.Stats()
        req, self._req = self._req, None
        L.check(L.lib().shine_wait(req, C.byref(st)))
        self._res.stats = st.as_dict()
        return self._res


class Index:
    def __init__(self, handle: int, dim: int, metric: int):
        self._h = C.c_void_p(handle)
        self.dim = dim
        self.metric = metric
        self.mode = L.MODE_EXACT

    # ---- construction ----------------------------------------------------------------------------------
    @classmethod
    def open(cls, dump_paths, dim: int, M: int, metric: int = L.METRIC_L2, elem: int = L.ELEM_F32, gpus=None,
             placement: str = "replica", cache: float = 0.0):
        """placement "replica": every GPU holds the whole index; "sharded": memory node s lives on GPU slot
        s % len(gpus) only and the others read it over xGMI (include/shine_gpu.h, SHINE_PLACE_SHARDED).
        cache (sharded): share of every other slot's records, hottest first, each GPU keeps local copies of."""
        arr = (C.c_char_p * len(dump_paths))(*[str(p).encode() for p in dump_paths])
        g, ng = _gpus(gpus)
        h = C.c_void_p()
        L.check(L.lib().shine_open_ex(arr, len(dump_paths), dim, M, metric, elem, g, ng, _placement(placement),
                                      float(cache), C.byref(h)))
        return cls(h.value, dim, metric)

    @classmethod
    def from_buffers(cls, dumps, dim: int, M: int, metric: int = L.METRIC_L2, elem: int = L.ELEM_F32, gpus=None,
                     placement: str = "replica", cache: float = 0.0):
        dumps, ptrs, sizes = _dump_arrays(dumps)
        g, ng = _gpus(gpus)
        h = C.c_void_p()
        L.check(L.lib().shine_open_buffers_ex(ptrs, sizes, len(dumps), dim, M, metric, elem, g, ng,
                                              _placement(placement), float(cache), C.byref(h)))
        return cls(h.value, dim, metric)

    def close(self):
        if self._h is not None and self._h.value:
            L.check(L.lib().shine_close(self._h))
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        inf = L.IndexInfo()
        L.check(L.lib().shine_index_get_info(self._h, C.byref(inf)))
        return inf.as_dict()

    def set_search_mode(self, mode: int) -> None:
        """L.MODE_EXACT (reference heap order, tie-exact) or L.MODE_FAST (sorted list, ascending results)."""
        L.check(L.lib().shine_set_search_mode(self._h, mode))
        self.mode = mode

    # ---- queries -----------------------------------------------------------------------------------------
    def set_cache_policy(self, policy: int, ratio_percent: float = 5.0, seed: int = 0) -> None:
        """SHINE_CACHE_STATIC / SHINE_CACHE_DYNAMIC (include/shine_gpu.h): the reference's runtime admission and
        cooling-table eviction, applied between calls, ratio_percent % of the estimated index size per GPU."""
        L.check(L.lib().shine_set_cache_policy(self._h, int(policy), float(ratio_percent), int(seed)))

    def cache_update(self) -> None:
        L.check(L.lib().shine_cache_update(self._h))

    def cache_wait(self) -> None:
        """Wait for the pipelined replay of the last call's logs (shine_cache_wait) and enqueue its updates."""
        L.check(L.lib().shine_cache_wait(self._h))

    def cache_keys(self, slot: int) -> np.ndarray:
        """uids the dynamic cache of GPU slot `slot` holds, ascending."""
        n = C.c_uint64()
        L.check(L.lib().shine_cache_keys(self._h, slot, None, 0, C.byref(n)))
        out = np.empty(n.value, dtype=np.uint32)
        L.check(L.lib().shine_cache_keys(self._h, slot, _ptr(out), out.size, C.byref(n)))
        return out

    def device_ids(self, uids: np.ndarray) -> np.ndarray:
        u = np.ascontiguousarray(uids, dtype=np.uint32)
        out = np.empty_like(u)
        L.check(L.lib().shine_device_ids(self._h, _ptr(u), u.size, _ptr(out)))
        return out

    def knn(self, queries: np.ndarray, k: int, ef: int, query_ids: np.ndarray | None = None) -> KnnResult:
        """shine_knn_batch_ex (shine_knn_batch plus per-query counters): query i is answered on GPU slot query_ids[i] % n_gpus (position when None)."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be (nq, {self.dim})")
        nq = q.shape[0]
        qid = None if query_ids is None else np.ascontiguousarray(query_ids, dtype=np.uint32)
        if qid is not None and qid.shape != (nq,):
            raise ValueError("query_ids must hold one id per query")
        ids = np.empty((nq, k), dtype=np.uint32)
        dists = np.empty((nq, k), dtype=np.float32)
        qs = np.empty((nq, L.QS_WORDS), dtype=np.uint32)
        st = L.Stats()
        L.check(L.lib().shine_knn_batch_ex(self._h, _ptr(q), _ptr(qid), nq, k, ef, _ptr(ids), _ptr(dists), _ptr(qs),
                                        C.byref(st)))
        return KnnResult(ids, dists, qs, st.as_dict())

    def knn_async(self, queries: np.ndarray, k: int, ef: int, query_ids: np.ndarray | None = None) -> "KnnRequest":
        """shine_knn_batch_async: enqueue and return at once; KnnRequest.wait() (shine_wait) gives the KnnResult.
        Several requests may be in flight on one handle; each is waited for once."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be (nq, {self.dim})")
        nq = q.shape[0]
        qid = None if query_ids is None else np.ascontiguousarray(query_ids, dtype=np.uint32)
        if qid is not None and qid.shape != (nq,):
            raise ValueError("query_ids must hold one id per query")
        res = KnnResult(np.empty((nq, k), dtype=np.uint32), np.empty((nq, k), dtype=np.float32),
                        np.empty((nq, L.QS_WORDS), dtype=np.uint32), {})
        req = C.c_void_p()
        L.check(L.lib().shine_knn_batch_async(self._h, _ptr(q), _ptr(qid), nq, k, ef, _ptr(res.ids), _ptr(res.dists),
                                              _ptr(res.qstats), C.byref(req)))
        return KnnRequest(req, res)

    def prepare(self, nq: int, k: int, ef: int) -> None:
        """shine_prepare: one-time setup (streams, scratch, staging, kernel code) for calls of up to nq queries."""
        L.check(L.lib().shine_prepare(self._h, nq, k, ef))

    def cache_warmup(self, queries: np.ndarray, k: int, ef: int, query_ids: np.ndarray | None = None) -> None:
        """shine_cache_warmup: run the warmup split and re-rank every stripe's cached prefix by its reads."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        qid = None if query_ids is None else np.ascontiguousarray(query_ids, dtype=np.uint32)
        L.check(L.lib().shine_cache_warmup(self._h, _ptr(q), _ptr(qid), q.shape[0], k, ef))

    def release_stream(self, stream: int) -> None:
        """shine_release_stream: wait for `stream` and drop the handle's scratch for it."""
        L.check(L.lib().shine_release_stream(self._h, C.c_void_p(stream)))

    def knn_device(self, q_ptr: int, nq: int, k: int, ef: int, ids_ptr: int, dists_ptr: int | None,
                   qstats_ptr: int | None, stream: int | None = None, gpu_slot: int = 0) -> None:
        L.check(L.lib().shine_knn_batch_device(self._h, gpu_slot, C.c_void_p(q_ptr), nq, k, ef, C.c_void_p(ids_ptr),
                                               C.c_void_p(dists_ptr) if dists_ptr else None,
                                               C.c_void_p(qstats_ptr) if qstats_ptr else None,
                                               C.c_void_p(stream) if stream else None))

    def distance_device(self, q_ptr: int, nq: int, uids_ptr: int, n_per: int, out_ptr: int,
                        stream: int | None = None, gpu_slot: int = 0) -> None:
        L.check(L.lib().shine_distance_batch_device(self._h, gpu_slot, C.c_void_p(q_ptr), nq, C.c_void_p(uids_ptr),
                                                    n_per, C.c_void_p(out_ptr),
                                                    C.c_void_p(stream) if stream else None))

    def route(self, queries: np.ndarray) -> np.ndarray:
        """GPU slot of every query of a batch (shine_route): id % n_gpus, or the nearest region with room."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        out = np.empty(q.shape[0], dtype=np.uint32)
        L.check(L.lib().shine_route(self._h, _ptr(q), q.shape[0], _ptr(out)))
        return out

    def algorithmic_bytes(self, qstats: np.ndarray) -> int:
        qs = np.ascontiguousarray(qstats, dtype=np.uint32)
        return int(L.lib().shine_algorithmic_bytes(self._h, _ptr(qs), qs.shape[0]))


def build(base: np.ndarray, M: int, ef_construction: int, metric: int = L.METRIC_L2, n_shards: int = 1,
          seed: int = 1234, threads: int = 0) -> tuple[list[np.ndarray], int]:
    """Parallel HNSW::insert over base[0..n) (ids = positions).  Returns (dump images, build distcomps)."""
    b = np.ascontiguousarray(base, dtype=np.float32)
    h = C.c_void_p()
    L.check(L.lib().shine_build(_ptr(b), b.shape[0], b.shape[1], M, ef_construction, metric, n_shards, seed,
                                threads, C.byref(h)))
    try:
        dumps = []
        for s in range(n_shards):
            n = L.lib().shine_build_dump_size(h, s)
            p = L.lib().shine_build_dump_data(h, s)
            dumps.append(np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n,)).copy())
        dc = int(L.lib().shine_build_distcomps(h))
    finally:
        L.lib().shine_build_free(h)
    return dumps, dc


class GpuBuild:
    """shine_gpu_build: the GPU batch builder (HNSW::insert on one MI355X, include/shine_gpu.h).  `base` is a numpy
    array (host rows) or an integer device pointer to n x dim f32 rows on GPU `gpu` (then n and dim are required).
    Use `open()` for a search handle over the built graph, `dumps()` for the reference's dump images."""

    def __init__(self, base, M: int, ef_construction: int, metric: int = L.METRIC_L2, seed: int = 1234, gpu: int = 0,
                 n: int | None = None, dim: int | None = None, batch_fraction: float = 0.0, max_batch: int = 0):
        self._h = C.c_void_p()
        if isinstance(base, np.ndarray):
            b = np.ascontiguousarray(base, dtype=np.float32)
            n, dim = b.shape
            ptr, on_dev = _ptr(b), 0
        else:
            if n is None or dim is None:
                raise ValueError("a device pointer needs n and dim")
            ptr, on_dev = C.c_void_p(int(base)), 1
        self.n, self.dim, self.M, self.efc = int(n), int(dim), M, ef_construction
        L.check(L.lib().shine_gpu_build(ptr, on_dev, self.n, self.dim, M, ef_construction, metric, seed, gpu,
                                        float(batch_fraction), int(max_batch), C.byref(self._h)))
        self.metric = metric

    def stats(self) -> dict:
        st = L.GpuBuildStats()
        L.check(L.lib().shine_gpu_build_get_stats(self._h, C.byref(st)))
        return st.as_dict()

    def dumps(self, n_shards: int = 1, copy: bool = True) -> list[np.ndarray]:
        """The dump images of n_shards memory nodes.  copy=False: views of the build's own host buffers (no second
        copy of a 60 GB index), valid until the next dumps() call or close()."""
        L.check(L.lib().shine_gpu_build_dumps(self._h, n_shards))
        out = []
        for s in range(n_shards):
            n = L.lib().shine_gpu_build_dump_size(self._h, s)
            p = L.lib().shine_gpu_build_dump_data(self._h, s)
            v = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n,))
            out.append(v.copy() if copy else v)
        return out

    def write(self, directory: str) -> None:
        L.check(L.lib().shine_gpu_build_write(self._h, str(directory).encode()))

    def open(self, elem: int = L.ELEM_F32) -> "Index":
        h = C.c_void_p()
        L.check(L.lib().shine_gpu_build_open(self._h, elem, C.byref(h)))
        return Index(h.value, self.dim, self.metric)

    def open_ex(self, n_shards: int = 1, elem: int = L.ELEM_F32, gpus=None, placement: str = "replica",
                cache: float = 0.0) -> "Index":
        """shine_gpu_build_open_ex: any placement (e.g. sharded over GPU slots), the records on n_shards memory nodes
        as dumps(n_shards) would put them; the build keeps its arrays."""
        g, ng = _gpus(gpus)
        h = C.c_void_p()
        L.check(L.lib().shine_gpu_build_open_ex(self._h, n_shards, elem, g, ng, _placement(placement), float(cache),
                                                C.byref(h)))
        return Index(h.value, self.dim, self.metric)

    def close(self):
        if self._h is not None and self._h.value:
            L.lib().shine_gpu_build_free(self._h)
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan_regions(dumps, dim: int, M: int, metric: int, k: int) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Host-only region planner of SHINE_PLACE_SHARDED_REGIONS: fetch_level(500) + balanced k-means.
    Returns (centroids [k or 2k, dim], region of every uid, region of every centroid)."""
    dumps, ptrs, sizes = _dump_arrays(dumps)
    cent = np.empty((2 * k, dim), dtype=np.float32)
    mapping = np.empty(2 * k, dtype=np.uint32)
    nc = C.c_uint32(0)
    n_uid = _max_uid(dumps, dim, M) + 1
    region = np.full(n_uid, 0xFFFFFFFF, dtype=np.uint32)
    L.check(L.lib().shine_plan_regions(ptrs, sizes, len(dumps), dim, M, metric, k, _ptr(region), n_uid, _ptr(cent),
                                       _ptr(mapping), C.byref(nc)))
    return cent[:nc.value].copy(), region, mapping[:nc.value].copy()


def kmeans(rows: np.ndarray, k: int, metric: int = L.METRIC_L2, balanced: bool = True) -> dict:
    """Kmeans<Distance> over rows (shine_kmeans): run_and_optimize (balanced) or run_kmeans.  Returns centroids
    [k or 2k, dim], mapping (centroid -> region), region sizes and the Lloyd / balancing iteration counts."""
    x = np.ascontiguousarray(rows, dtype=np.float32)
    n, dim = x.shape
    cent = np.empty((2 * k, dim), dtype=np.float32)
    mapping = np.empty(2 * k, dtype=np.uint32)
    sizes = np.zeros(k, dtype=np.uint64)
    nc = C.c_uint32(0)
    it = np.zeros(2, dtype=np.uint32)
    L.check(L.lib().shine_kmeans(_ptr(x), n, dim, metric, k, int(balanced), _ptr(cent), _ptr(mapping), C.byref(nc),
                                 _ptr(sizes), _ptr(it)))
    return {"centroids": cent[:nc.value].copy(), "mapping": mapping[:nc.value].copy(), "sizes": sizes,
            "iterations": int(it[0]), "balance_iterations": int(it[1])}


def router_run(centroids: np.ndarray, mapping: np.ndarray, k: int, queries: np.ndarray, metric: int = L.METRIC_L2,
               queue_sizes: np.ndarray | None = None, adaptive: bool = True) -> tuple[np.ndarray, np.ndarray]:
    """QueryRouter::run_routing's region per query (shine_router_run); queue_sizes[b] are the queue sizes at batch
    boundary b (the last row repeats).  Returns (region per query, limits after the last boundary)."""
    c = np.ascontiguousarray(centroids, dtype=np.float32)
    m = np.ascontiguousarray(mapping, dtype=np.uint32)
    q = np.ascontiguousarray(queries, dtype=np.float32)
    qs = None if queue_sizes is None else np.ascontiguousarray(queue_sizes, dtype=np.uint32).reshape(-1, k)
    out = np.empty(q.shape[0], dtype=np.uint32)
    lim = np.zeros(k, dtype=np.uint64)
    L.check(L.lib().shine_router_run(_ptr(c), _ptr(m), c.shape[0], k, c.shape[1], metric, _ptr(q), q.shape[0],
                                     None if qs is None else _ptr(qs), 0 if qs is None else qs.shape[0], int(adaptive),
                                     _ptr(out), _ptr(lim)))
    return out, lim


def plan_sharded_views(gpus, stride_bytes: int, cached_bytes: int = 0) -> dict:
    """Host-only view plan of SHINE_PLACE_SHARDED (shine_plan_sharded_views; the plan shine_open_ex maps).
    Returns {"pieces": [dict per piece], "access": [[devices] per view], "peer_pairs": [(a, b), ...]}."""
    g = (C.c_int * len(gpus))(*gpus)
    G = len(gpus)
    n = C.c_uint64()
    L.check(L.lib().shine_plan_sharded_views(g, G, stride_bytes, cached_bytes, None, 0, C.byref(n), None, None, None,
                                             None))
    pieces = (L.ViewPiece * max(1, n.value))()
    access = np.zeros(G * G, np.int32)
    n_access = np.zeros(G, np.uint32)
    pairs = np.zeros(2 * G * G, np.int32)
    n_pairs = C.c_uint32()
    L.check(L.lib().shine_plan_sharded_views(g, G, stride_bytes, cached_bytes, C.cast(pieces, C.c_void_p), n.value,
                                             C.byref(n), _ptr(access), _ptr(n_access), _ptr(pairs), C.byref(n_pairs)))
    out = [{k: getattr(pieces[i], k) for k, _ in L.ViewPiece._fields_} for i in range(n.value)]
    acc = [access[o * G:o * G + int(n_access[o])].tolist() for o in range(G)]
    pp = [(int(pairs[2 * i]), int(pairs[2 * i + 1])) for i in range(n_pairs.value)]
    return {"pieces": out, "access": acc, "peer_pairs": pp}


def graph_stats(dumps, dim: int, M: int) -> dict:
    """Host-only reachability diagnostics of an index (shine_graph_stats_buffers)."""
    dumps, ptrs, sizes = _dump_arrays(dumps)
    st = L.GraphStats()
    L.check(L.lib().shine_graph_stats_buffers(ptrs, sizes, len(dumps), dim, M, C.byref(st)))
    return st.as_dict()


def _max_uid(dumps, dim: int, M: int) -> int:
    """Largest uid in the dumps (record walk of memory_node.hh:15-27 / node.hh:10-19)."""
    best = 0
    for d in dumps:
        free = int(np.frombuffer(d[:8].tobytes(), np.uint64)[0])
        off = 16
        while off < free:
            uid, level = np.frombuffer(d[off + 8:off + 16].tobytes(), np.uint32)
            best = max(best, int(uid))
            size = 16 + 4 * dim + 4 + 8 * 2 * M + int(level) * (4 + 8 * M)
            off += size + (-size) % 8
    return best


def dump_name(M: int, efc: int, i: int, n: int) -> str:
    """compute_node.cc:428-430"""
    return f"index_m{M}_efc{efc}_node{i + 1}_of{n}.dat"
