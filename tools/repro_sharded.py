import sys, time
sys.path.insert(0, "dm-hnsw-reference_amd"); sys.path.insert(0, ".")
import numpy as np
import shine_amd
from shine_amd import datasets as D
from bench import host_threads
use_torch = len(sys.argv) > 1 and sys.argv[1] == "torch"
if use_torch:
    import torch
    x = torch.empty(int(2e9), dtype=torch.uint8, device="cuda")
for n, shards, gpus in [(20000, 4, [0, 0]), (200000, 4, [0, 0]), (1000000, 4, [0, 0]), (1000000, 2, [0, 0]), (1000000, 4, [0, 0, 0, 0])]:
    base = D.sift_like(n, seed=1)
    t = time.time()
    dumps, _ = shine_amd.build(base, 16, 64, 0, shards, seed=5, threads=host_threads())
    try:
        with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=gpus, placement="sharded") as idx:
            inf = idx.info()
            r = idx.knn(D.sift_like(64, seed=2), 10, 64)
            print("ok", n, shards, gpus, inf["id_space"], inf["device_bytes"], r.qstats[:, 6].max(), f"{time.time()-t:.1f}s", flush=True)
    except Exception as e:
        print("FAIL", n, shards, gpus, e, flush=True)
