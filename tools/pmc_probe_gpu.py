"""Diagnostics: a few search batches on a GPU-built index, for rocprofv3 --pmc passes (one pass per process; the
counters of every dispatch land in the pass's CSV and tools/pmc.py / pmc_summary.py keep the search kernel's).

  WORKLOAD=sift1m    the bench's index: SIFT-shaped 1M x 128, L2, M=16, efC=200 (bench.py --builder gpu), ef 128
  WORKLOAD=cfg5_10m  TTI-shaped 10M x 200, inner product, fp16 rows, Zipf(1.0) query mix, ef 250 (N: another size,
                     e.g. N=50000000 for cfg 5's full size)
ROWS=f32|u8|f16 (default: the workload's), MODE=fast|exact, EF, NQ (queries per batch, default 1024), REPS.
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
import torch  # noqa: E402
import shine_amd  # noqa: E402
from shine_amd import datasets as D  # noqa: E402

L = shine_amd._lib
work = os.environ.get("WORKLOAD", "sift1m")
nq = int(os.environ.get("NQ", "1024"))
if work == "sift1m":
    base = torch.from_numpy(D.sift_like(1_000_000, seed=1)).cuda()
    q = D.sift_like(nq, seed=2)
    dim, metric, ef, rows = 128, 0, 128, os.environ.get("ROWS", "f32")
else:
    base = D.generate_device("tti_like", int(os.environ.get("N", "10000000")), seed=1, d=200)
    pool = D.generate_device("tti_like", 500_000, seed=2, d=200).cpu().numpy()
    q = np.ascontiguousarray(D.zipf_query_mix(pool, nq, 1.0, seed=3)[0])
    dim, metric, ef, rows = 200, 1, 250, os.environ.get("ROWS", "f16")
ef = int(os.environ.get("EF", str(ef)))
gb = shine_amd.GpuBuild(base.data_ptr(), 16, 200, metric, seed=1234, n=base.shape[0], dim=dim)
del base
torch.cuda.empty_cache()
elem = {"f32": L.ELEM_F32, "f16": L.ELEM_F16, "u8": L.ELEM_U8}[rows]
idx = gb.open(elem)
gb.close()
idx.set_search_mode(L.MODE_FAST if os.environ.get("MODE", "fast") == "fast" else L.MODE_EXACT)
for _ in range(int(os.environ.get("REPS", "3"))):
    r = idx.knn(q, 10, ef)
print("kernel_ms", r.stats["kernel_ms"], "distcomps", r.qstats[:, 0].mean(), "L0 lists", r.qstats[:, 4].mean())
