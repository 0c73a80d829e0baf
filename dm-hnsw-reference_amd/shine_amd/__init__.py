"""shine_amd — MI355X-native SHINE compute-node query engine (host-side Python mirror of the C ABI)."""
from . import _lib
from ._lib import (ELEM_AUTO, ELEM_F16, ELEM_F32, ELEM_I8, ELEM_U8, METRIC_IP, METRIC_L2, QS_DISTCOMPS, QS_LISTS_L0, QS_LISTS_UPPER,
                   QS_MAX_NEXT, QS_NRESULT, QS_STATUS, QS_TIES, QS_VISITED_L0, QS_VISITED_UPPER, QS_WORDS, QS_REMOTE_VEC,
                   QS_REMOTE_LIST, QS_CACHED_VEC, QS_CACHED_LIST, MODE_EXACT,
                   MODE_FAST, PLACE_REPLICA, PLACE_SHARDED, PLACE_SHARDED_REGIONS, CACHE_STATIC, CACHE_DYNAMIC, ShineError)
from .index import (GpuBuild, Index, KnnResult, build, dump_name, graph_stats, kmeans, plan_regions, plan_sharded_views,
                    router_run)

__all__ = ["GpuBuild", "Index", "KnnResult", "build", "dump_name", "graph_stats", "kmeans", "plan_regions", "plan_sharded_views", "router_run", "ShineError", "PLACE_REPLICA", "PLACE_SHARDED",
           "PLACE_SHARDED_REGIONS", "METRIC_L2", "METRIC_IP", "ELEM_F32",
           "ELEM_F16", "ELEM_U8", "ELEM_I8", "ELEM_AUTO", "QS_DISTCOMPS", "QS_VISITED_UPPER", "QS_VISITED_L0", "QS_LISTS_UPPER", "QS_LISTS_L0",
           "QS_MAX_NEXT", "QS_TIES", "MODE_EXACT", "MODE_FAST", "QS_STATUS", "QS_NRESULT", "QS_WORDS", "QS_REMOTE_VEC",
           "QS_REMOTE_LIST", "QS_CACHED_VEC", "QS_CACHED_LIST", "CACHE_STATIC", "CACHE_DYNAMIC", "_lib"]
