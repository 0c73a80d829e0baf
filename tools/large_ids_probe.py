#!/usr/bin/env python3
"""Phase timing of tests/test_gpu_large_ids.py's workload (2^26 + 2^16 records of 16-d rows, GPU-built), with a
heartbeat line every 20 s: which phase costs what at this size (row generation, the GPU build, the dump images, the
oracle, the searches)."""
from __future__ import annotations

import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

T0 = time.time()
PHASE = ["start"]


def log(msg):
    print(f"[large ids probe {time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def heartbeat():
    while True:
        time.sleep(20)
        log(f"... in phase {PHASE[0]}")


def phase(name):
    PHASE[0] = name
    log(f"begin {name}")


def main():
    threading.Thread(target=heartbeat, daemon=True).start()
    phase("import torch")
    import torch
    torch.cuda.init()
    phase("import shine_amd / oracle")
    import oracle as O
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 26) + (1 << 16)
    dim, M, efc, ef, k = 16, 8, 24, 64, 10
    phase(f"generate {n} x {dim}")
    base_t = D.generate_device("deep_like", n, seed=61, d=dim)
    torch.cuda.synchronize()
    q = D.generate_device("deep_like", 64, seed=62, d=dim).cpu().numpy()
    phase("GPU build")
    gb = shine_amd.GpuBuild(base_t.data_ptr(), M, efc, L.METRIC_L2, seed=7, n=n, dim=dim)
    log(f"build stats {gb.stats()}")
    del base_t
    torch.cuda.empty_cache()
    phase("dump images")
    dumps = gb.dumps(1, copy=False)
    log(f"dump bytes {sum(d.size for d in dumps)}")
    phase("oracle open + knn")
    ref = O.OracleIndex(dumps, dim, M, L.METRIC_L2).knn(q, k, ef, threads=8)
    del dumps
    phase("open + search")
    import os
    os.environ["SHINE_DEBUG_VISCAP"] = "64"
    os.environ["SHINE_DEBUG_VIS16"] = "0"
    with gb.open() as idx:
        for mode in (L.MODE_EXACT, L.MODE_FAST):
            idx.set_search_mode(mode)
            r = idx.knn(q, k, ef)
            log(f"mode {mode}: same ids as oracle {(r.ids == ref[0]).all(1).mean():.3f}, visited mean "
                f"{r.qstats[:, 2].mean():.0f}, retries {r.stats['overflow_retries']}")
    gb.close()
    phase("done")


if __name__ == "__main__":
    main()
