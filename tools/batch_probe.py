"""Diagnostics: search-kernel time vs batch size on the phase-profile index (tools/phase_profile.py builds it).

A latency-bound kernel keeps its launch time flat while the batch grows up to the point where the chip's
wave slots fill; the knee says how much concurrency one batch leaves unused.
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
import shine_amd  # noqa: E402
from shine_amd import datasets as D  # noqa: E402

path = Path("/tmp/shine_bench_phase") / "dump" / shine_amd.dump_name(16, 200, 0, 1)
if not path.exists():  # the same index tools/phase_profile.py builds
    dumps, _ = shine_amd.build(D.sift_like(1_000_000, seed=1), 16, 200, 0, 1, 1234,
                               threads=int(os.environ.get("OMP_NUM_THREADS", "16")))
    path.parent.mkdir(parents=True, exist_ok=True)
    dumps[0].tofile(path)
q = D.sift_like(16384, seed=2)
idx = shine_amd.Index.open([path], 128, 16, 0, gpus=[0])
for mode in (shine_amd.MODE_FAST, shine_amd.MODE_EXACT):
    idx.set_search_mode(mode)
    for nq in (64, 256, 512, 1024, 2048, 4096, 8192, 16384):
        ts = []
        for rep in range(3):
            r = idx.knn(q[:nq], 10, int(os.environ.get("EF", "128")))
            ts.append(r.stats["kernel_ms"])
        t = min(ts)
        print(f"mode {mode} nq {nq:6d} kernel {t:8.3f} ms  {nq / t * 1e3 / 1e6:6.3f} MQPS  "
              f"L0 lists mean {r.qstats[:, 4].mean():.1f} max {r.qstats[:, 4].max()}", flush=True)
