"""Diagnostics: the two-wavefront fast kernel (SHINE_DUO=1) on a small index, against the one-wavefront kernel."""
import os
import sys
sys.path.insert(0, "dm-hnsw-reference_amd")
import numpy as np
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

base = D.sift_like(20000, seed=5)
q = D.sift_like(300, seed=6)
dumps, _ = shine_amd.build(base, 16, 100, 0, 1, seed=3, threads=8)
out = {}
for duo in ("0", "1"):
    if duo == "1":
        os.environ["SHINE_DUO"] = "1"
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        idx.set_search_mode(L.MODE_FAST)
        out[duo] = idx.knn(q, 10, 128)
    print("duo", duo, "done", out[duo].stats["kernel_ms"], flush=True)
a, b = out["0"], out["1"]
print("ids equal", np.array_equal(a.ids, b.ids), "qstats equal", np.array_equal(a.qstats, b.qstats), flush=True)
