"""Diagnostics: per-phase shader-clock shares of the search kernel on the bench's SIFT1M-shaped index.

Runs the PROF kernel variant (SHINE_PHASE_PROFILE=1, s_memtime stamps; its run time is not quoted) on one
1,024-query batch and prints the share of wave-cycles per phase of the expansion loop.
"""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
import shine_amd  # noqa: E402
from shine_amd import datasets as D  # noqa: E402

n = int(os.environ.get("N", "1000000"))
ef = int(os.environ.get("EF", "128"))
cache = Path("/tmp/shine_bench_phase") if n == 1_000_000 else Path(f"/tmp/shine_size_probe/n{n}")
path = (cache / "dump" if n == 1_000_000 else cache) / shine_amd.dump_name(16, 200, 0, 1)
if not path.exists():
    base = D.sift_like(n, seed=1)
    t = time.time()
    dumps, _ = shine_amd.build(base, 16, 200, 0, 1, 1234, threads=int(os.environ.get("OMP_NUM_THREADS", "16")))
    print(f"built in {time.time() - t:.1f}s", file=sys.stderr)
    path.parent.mkdir(parents=True, exist_ok=True)
    dumps[0].tofile(path)
q = D.sift_like(1024, seed=2)
elem = shine_amd.ELEM_U8 if os.environ.get("ROWS") == "u8" else shine_amd.ELEM_F32  # ROWS=u8: byte rows
idx = shine_amd.Index.open([path], 128, 16, 0, elem=elem, gpus=[0])
if os.environ.get("MODE", "exact") == "fast":
    idx.set_search_mode(shine_amd.MODE_FAST)
r = idx.knn(q, 10, ef)
print("plain kernel_ms", r.stats["kernel_ms"], file=sys.stderr)
os.environ["SHINE_PHASE_PROFILE"] = "1"
r = idx.knn(q, 10, ef)
print("profiled kernel_ms", r.stats["kernel_ms"], "mean distcomps", r.qstats[:, 0].mean(), "mean L0 lists",
      r.qstats[:, 4].mean(), "mean max next", r.qstats[:, 5].mean(), file=sys.stderr)
