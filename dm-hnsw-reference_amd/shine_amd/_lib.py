"""ctypes binding of libshine_gpu.so (include/shine_gpu.h).

The library is the product: there is no fallback.  If it is missing or fails to load, every entry point
raises ShineError — a GPU box without the HIP extension must fail loudly, never run something else.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # dm-hnsw-reference_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = Path(os.environ.get("SHINE_GPU_LIB", PKG_ROOT / "libshine_gpu.so"))
HEADER = REPO_ROOT / "include" / "shine_gpu.h"

OK, ERR_ARG, ERR_IO, ERR_FORMAT, ERR_HIP, ERR_NOMEM, ERR_OVERFLOW = range(7)
METRIC_L2, METRIC_IP = 0, 1
ELEM_F32, ELEM_F16, ELEM_U8, ELEM_I8, ELEM_AUTO = 0, 1, 2, 3, 4
QS_DISTCOMPS, QS_VISITED_UPPER, QS_VISITED_L0, QS_LISTS_UPPER, QS_LISTS_L0, QS_MAX_NEXT, QS_STATUS, QS_NRESULT = range(8)
QS_REMOTE_VEC, QS_REMOTE_LIST, QS_CACHED_VEC, QS_CACHED_LIST = range(8, 12)
QS_WORDS = 12
QS_TIES = 5  # fast mode's meaning of word 5
MODE_EXACT, MODE_FAST = 0, 1
CACHE_STATIC, CACHE_DYNAMIC = 0, 1
PLACE_REPLICA, PLACE_SHARDED, PLACE_SHARDED_REGIONS = 0, 1, 2


class ShineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"shine error {code}: {msg}")
        self.code = code


class Stats(C.Structure):
    _fields_ = [
        ("processed", C.c_uint64),
        ("distcomps", C.c_uint64),
        ("visited_nodes", C.c_uint64),
        ("visited_nodes_l0", C.c_uint64),
        ("visited_neighborlists", C.c_uint64),
        ("visited_neighborlists_l0", C.c_uint64),
        ("rdma_reads_in_bytes", C.c_uint64),
        ("algorithmic_bytes", C.c_uint64),
        ("overflow_retries", C.c_uint64),
        ("remote_reads_in_bytes", C.c_uint64),
        ("cache_hits", C.c_uint64),
        ("cache_misses", C.c_uint64),
        ("kernel_ms", C.c_double),
        ("node_reads", C.c_uint64),
        ("node_cache_hits", C.c_uint64),
        ("cache_admitted", C.c_uint64),
        ("cache_evicted", C.c_uint64),
        ("cache_rescued", C.c_uint64),
        ("cache_log_dropped", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class IndexInfo(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint64),
        ("num_upper_rows", C.c_uint64),
        ("device_bytes", C.c_uint64),
        ("dim", C.c_uint32),
        ("M", C.c_uint32),
        ("metric", C.c_uint32),
        ("elem", C.c_uint32),
        ("max_level", C.c_uint32),
        ("entry_uid", C.c_uint32),
        ("n_shards", C.c_uint32),
        ("n_gpus", C.c_uint32),
        ("placement", C.c_uint32),
        ("reserved0", C.c_uint32),
        ("id_space", C.c_uint64),
        ("cache_fraction", C.c_double),
        ("cus", C.c_uint32),
        ("lds_per_cu", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class GraphStats(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint64),
        ("reachable_l0", C.c_uint64),
        ("reachable_any", C.c_uint64),
        ("zero_indegree_l0", C.c_uint64),
        ("full_lists_l0", C.c_uint64),
        ("mean_degree_l0", C.c_double),
        ("max_level", C.c_uint32),
        ("reserved0", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved0"}


class GpuBuildStats(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint64),
        ("num_upper_rows", C.c_uint64),
        ("batches", C.c_uint64),
        ("upper_lists", C.c_uint64),
        ("requests", C.c_uint64),
        ("rows_appended", C.c_uint64),
        ("rows_pruned", C.c_uint64),
        ("pools_truncated", C.c_uint64),
        ("upper_beams_stopped", C.c_uint64),
        ("search_failures", C.c_uint64),
        ("distcomps", C.c_uint64),
        ("max_level", C.c_uint32),
        ("entry_uid", C.c_uint32),
        ("ms_total", C.c_double),
        ("ms_search", C.c_double),
        ("ms_upper", C.c_double),
        ("ms_select", C.c_double),
        ("ms_sort", C.c_double),
        ("ms_prune", C.c_double),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class ViewPiece(C.Structure):
    _fields_ = [
        ("view_slot", C.c_uint32),
        ("stripe", C.c_uint32),
        ("offset", C.c_uint64),
        ("size", C.c_uint64),
        ("backing_device", C.c_int32),
        ("kind", C.c_uint32),
    ]


VIEW_OWN, VIEW_COPY, VIEW_PEER = 0, 1, 2

P = C.c_void_p
U32, U64, I32 = C.c_uint32, C.c_uint64, C.c_int
PU8 = C.POINTER(C.c_uint8)

# name -> (restype, argtypes); must cover every function include/shine_gpu.h declares
PROTOTYPES = {
    "shine_open": (I32, [C.POINTER(C.c_char_p), U32, U32, U32, I32, I32, C.POINTER(I32), U32, C.POINTER(P)]),
    "shine_open_buffers": (I32, [C.POINTER(PU8), C.POINTER(U64), U32, U32, U32, I32, I32, C.POINTER(I32), U32,
                                 C.POINTER(P)]),
    "shine_open_ex": (I32, [C.POINTER(C.c_char_p), U32, U32, U32, I32, I32, C.POINTER(I32), U32, I32, C.c_double,
                            C.POINTER(P)]),
    "shine_open_buffers_ex": (I32, [C.POINTER(PU8), C.POINTER(U64), U32, U32, U32, I32, I32, C.POINTER(I32), U32, I32,
                                    C.c_double, C.POINTER(P)]),
    "shine_knn_batch": (I32, [P, P, P, U32, U32, U32, P, P, C.POINTER(Stats)]),  # SURVEY.md §8b's 9 arguments
    "shine_knn_batch_ex": (I32, [P, P, P, U32, U32, U32, P, P, P, C.POINTER(Stats)]),
    "shine_prepare": (I32, [P, U32, U32, U32]),
    "shine_knn_batch_async": (I32, [P, P, P, U32, U32, U32, P, P, P, C.POINTER(P)]),
    "shine_wait": (I32, [P, C.POINTER(Stats)]),
    "shine_release_stream": (I32, [P, P]),
    "shine_set_cache_policy": (I32, [P, I32, C.c_double, U64]),
    "shine_cache_update": (I32, [P]),
    "shine_cache_wait": (I32, [P]),
    "shine_cache_keys": (I32, [P, U32, P, U64, C.POINTER(U64)]),
    "shine_device_ids": (I32, [P, P, U32, P]),
    "shine_selftest_cache": (I32, [U32, U64, U32, P, P, P, P, P, U64, C.POINTER(U64), P]),
    "shine_cache_warmup": (I32, [P, P, P, U32, U32, U32]),
    "shine_knn_batch_device": (I32, [P, U32, P, U32, U32, U32, P, P, P, P]),
    "shine_distance_batch_device": (I32, [P, U32, P, U32, P, U32, P, P]),
    "shine_route": (I32, [P, P, U32, P]),
    "shine_plan_regions": (I32, [C.POINTER(PU8), C.POINTER(U64), U32, U32, U32, I32, U32, P, U64, P, P, P]),
    "shine_plan_sharded_views": (I32, [C.POINTER(I32), U32, U64, U64, P, U64, C.POINTER(U64), P, P, P,
                                       C.POINTER(U32)]),
    "shine_kmeans": (I32, [P, U64, U32, I32, U32, I32, P, P, P, P, P]),
    "shine_router_run": (I32, [P, P, U32, U32, U32, I32, P, U32, P, U32, I32, P, P]),
    "shine_set_search_mode": (I32, [P, I32]),
    "shine_index_get_info": (I32, [P, C.POINTER(IndexInfo)]),
    "shine_algorithmic_bytes": (U64, [P, P, U32]),
    "shine_close": (I32, [P]),
    "shine_selftest_heap": (I32, [I32, P, P, P, U32, U32, P, P, P]),
    "shine_last_error": (C.c_char_p, []),
    "shine_build_id": (C.c_char_p, []),
    "shine_graph_stats_buffers": (I32, [C.POINTER(PU8), C.POINTER(U64), U32, U32, U32, C.POINTER(GraphStats)]),
    "shine_build": (I32, [P, U64, U32, U32, U32, I32, U32, U32, U32, C.POINTER(P)]),
    "shine_build_dump_size": (U64, [P, U32]),
    "shine_build_dump_data": (P, [P, U32]),
    "shine_build_distcomps": (U64, [P]),
    "shine_build_write": (I32, [P, C.c_char_p, U32, U32]),
    "shine_build_free": (I32, [P]),
    "shine_gpu_build": (I32, [P, I32, U64, U32, U32, U32, I32, U32, I32, C.c_double, U32, C.POINTER(P)]),
    "shine_gpu_build_get_stats": (I32, [P, C.POINTER(GpuBuildStats)]),
    "shine_gpu_build_dumps": (I32, [P, U32]),
    "shine_gpu_build_dump_size": (U64, [P, U32]),
    "shine_gpu_build_dump_data": (P, [P, U32]),
    "shine_gpu_build_write": (I32, [P, C.c_char_p]),
    "shine_gpu_build_open": (I32, [P, I32, C.POINTER(P)]),
    "shine_gpu_build_open_ex": (I32, [P, U32, I32, C.POINTER(I32), U32, I32, C.c_double, C.POINTER(P)]),
    "shine_gpu_build_free": (I32, [P]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libshine_gpu.so once; raise ShineError if it is absent (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ShineError(ERR_HIP, f"{LIB_PATH} not built: run __graft_entry__.build() (make -C "
                                      f"dm-hnsw-reference_amd/csrc)")
        _one_hip_runtime()
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _one_hip_runtime() -> None:
    """One HIP runtime per process.  torch's ROCm libraries name the runtime `libamdhip64.so` (resolved in torch/lib),
    this library names `libamdhip64.so.7`: loaded first, ours would make torch load a second runtime next to it,
    and whichever initialises second finds no device.  Importing torch first lets the loader match our soname to
    torch's copy.  Without torch (e.g. the C façade) /opt/rocm's runtime is the only one."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def check(rc: int) -> None:
    if rc != OK:
        raise ShineError(rc, lib().shine_last_error().decode(errors="replace"))


def build_id() -> str:
    """The loaded library's provenance (shine_build_id): "src <source hash> git <head at build time>"."""
    return lib().shine_build_id().decode()


def source_hash() -> str:
    """The source hash the Makefile would compile into a library built from this tree (csrc/Makefile SRC_HASH)."""
    import hashlib
    csrc = PKG_ROOT / "csrc"
    names = sorted(p.name for p in csrc.iterdir() if p.is_file() and p.suffix in (".cc", ".h", ".hip"))
    h = hashlib.sha1()
    for path in [csrc / n for n in names] + [HEADER, csrc / "Makefile"]:
        h.update(path.read_bytes())
    return h.hexdigest()[:16]


def declared_symbols() -> list[str]:
    """Function names declared in include/shine_gpu.h (parsed from the header text)."""
    import re
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(shine_[a-z_0-9]+)\s*\(", text)))
