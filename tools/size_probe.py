"""Diagnostics: search-kernel time per level-0 expansion vs index size (L2- / MALL- / HBM-resident vectors).

Separates memory latency from in-wavefront work: with the index resident in a 4 MiB L2 the expansion time is
nearly all instruction latency; the growth up to the 1M-node (512 MB) index is the gather latency.
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

th = int(os.environ.get("OMP_NUM_THREADS", "16"))
q = D.sift_like(1024, seed=2)
for n in [int(x) for x in os.environ.get("SIZES", "5000,50000,300000,1000000").split(",")]:
    path = Path("/tmp/shine_size_probe") / f"n{n}" / shine_amd.dump_name(16, 200, 0, 1)
    if n == 1_000_000 and (Path("/tmp/shine_bench_phase") / "dump" / path.name).exists():
        path = Path("/tmp/shine_bench_phase") / "dump" / path.name
    if not path.exists():
        t = time.time()
        dumps, _ = shine_amd.build(D.sift_like(n, seed=1), 16, 200, 0, 1, 1234, threads=th)
        path.parent.mkdir(parents=True, exist_ok=True)
        dumps[0].tofile(path)
        print(f"built n={n} in {time.time() - t:.1f}s", flush=True)
    idx = shine_amd.Index.open([path], 128, 16, 0, gpus=[0])
    for mode in (shine_amd.MODE_FAST, shine_amd.MODE_EXACT):
        idx.set_search_mode(mode)
        for nq in (64, 1024):
            ts = []
            for rep in range(3):
                r = idx.knn(q[:nq], 10, 128)
                ts.append(r.stats["kernel_ms"])
            t = min(ts)
            lmax = r.qstats[:, 4].max()
            print(f"n {n:8d} mode {mode} nq {nq:5d} kernel {t:7.3f} ms  L0 lists mean {r.qstats[:, 4].mean():6.1f} "
                  f"max {lmax:4d}  -> {t * 1e3 / lmax:5.2f} us per expansion (slowest query)", flush=True)
    idx.close()
