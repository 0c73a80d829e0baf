"""Diagnostics: does a second batch in flight hide the fast kernel's tail?

Times K batches of the bench workload (SIFT1M-shaped, ef=128, batch 1024, fast mode) issued on one stream, then
the same K batches alternating over S streams of the same index handle (per-stream device scratch).  Prints QPS
per configuration and the per-query expansion-count distribution.
"""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
import shine_amd  # noqa: E402
from shine_amd import datasets as D  # noqa: E402

K = int(os.environ.get("K", "60"))
path = Path("/tmp/shine_overlap") / shine_amd.dump_name(16, 200, 0, 1)
if not path.exists():
    base = D.sift_like(1_000_000, seed=1)
    dumps, _ = shine_amd.build(base, 16, 200, 0, 1, 1234, threads=16)
    path.parent.mkdir(parents=True, exist_ok=True)
    dumps[0].tofile(path)
q = torch.from_numpy(D.sift_like(1024 * 10, seed=2)).cuda()
nb = 10
S = 4
idx = shine_amd.Index.open([path], 128, 16, 0, gpus=[0])
idx.set_search_mode(shine_amd.MODE_FAST)
streams = [torch.cuda.Stream() for _ in range(S)]
ids = torch.empty((nb, 1024, 10), dtype=torch.int32, device="cuda")
dd = torch.empty((nb, 1024, 10), dtype=torch.float32, device="cuda")
qs = torch.zeros((nb, 1024, 12), dtype=torch.int32, device="cuda")


def run(ns):
    for i in range(K + 5):
        if i == 5:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        b, s = i % nb, i % ns
        idx.knn_device(q[b * 1024:(b + 1) * 1024].data_ptr(), 1024, 10, 128, ids[b].data_ptr(), dd[b].data_ptr(),
                           qs[b].data_ptr(), stream=streams[s].cuda_stream)
    torch.cuda.synchronize()
    return K * 1024 / (time.perf_counter() - t0)


for ns in (1, 2, 3, 4, 1, 2):
    print(f"streams={ns}: {run(ns) / 1e6:.3f} M QPS", flush=True)
l0 = qs.cpu().numpy()[..., 4].reshape(-1).astype(float)
print("L0 lists per query: mean %.1f p50 %.0f p90 %.0f p99 %.0f max %.0f" % (l0.mean(), *np.percentile(l0, [50, 90, 99, 100])))
