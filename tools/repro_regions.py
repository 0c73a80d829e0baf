"""Diagnostics: region placement in a fresh process, then after a large partial-cache index was opened and closed."""
import sys
sys.path.insert(0, "dm-hnsw-reference_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
import numpy as np
import oracle as O
import shine_amd
from shine_amd import datasets as D

step = sys.argv[1]
base = D.sift_like(4000, seed=61)
q = D.sift_like(150, seed=62)
dumps, _, _ = O.build(base, 8, 48, 0, 4, seed=5)
ref_ids, _, _ = O.OracleIndex(dumps, 128, 8, 0).knn(q, k=10, ef=48)
if step == "after80k":
    b2 = D.sift_like(80000, seed=81)
    d2, _ = shine_amd.build(b2, 8, 40, 0, 2, seed=6, threads=8)
    with shine_amd.Index.from_buffers(d2, 128, 8, 0, gpus=[0, 0], placement="sharded", cache=0.5) as idx:
        idx.knn(D.sift_like(50, seed=1), 10, 40)
    print("80k open/close ok", flush=True)
for placement, cache in (("regions", 0.0), ("regions", 0.5)):
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0], placement=placement, cache=cache) as idx:
        print(placement, cache, idx.info()["id_space"], np.bincount(idx.route(q)), flush=True)
        r = idx.knn(q, 10, 48)
        print(placement, cache, "exact equal:", np.array_equal(r.ids, ref_ids), flush=True)
