#!/usr/bin/env python3
"""Where the host-to-host query phase loses time (diagnostics): bench index, fast mode, ef = 128.

Variants, each K steps of 1,024 queries over S streams (step i on stream i % S):
  full   pinned H2D of the queries -> knn -> D2H of ids and distances (bench.py value_host_to_host)
  h2d    pinned H2D -> knn
  d2h    knn on resident queries -> D2H
  none   knn only (the device value)
  zc     zero copy: the kernels read the queries from pinned host memory and write ids and distances into pinned
         host memory (mapped into the GPU's address space), so no copy engine and no cross-engine dependency
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

os.environ["GPU_MAX_HW_QUEUES"] = "8"  # as bench.py
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="none:4,full:4,zc:4,zc:2,zc:8")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--nbatches", type=int, default=24)
    p.add_argument("--out", default="")
    p.add_argument("--cache", default=os.environ.get("SHINE_BENCH_CACHE", "/tmp/shine_bench"))
    a = p.parse_args()
    import numpy as np
    import torch
    import shine_amd
    from shine_amd import datasets as D
    from bench import host_threads, log, prepare_dumps

    B, k, ef = 1024, 10, 128
    key = hashlib.sha1(f"{1_000_000}-128-16-200-1-sift_like-v3".encode()).hexdigest()[:12]
    paths = [Path(a.cache) / key / "dump" / shine_amd.dump_name(16, 200, 0, 1)]

    def build():
        base = D.sift_like(1_000_000, seed=1, d=128)
        dumps, _ = shine_amd.build(base, 16, 200, shine_amd.METRIC_L2, 1, seed=1234, threads=host_threads())
        return dumps

    prepare_dumps(paths, 0, None, build)
    idx = shine_amd.Index.open(paths, 128, 16, shine_amd.METRIC_L2, gpus=[0])
    idx.set_search_mode(shine_amd.MODE_FAST)
    qh = D.sift_like(B * a.nbatches, seed=2, d=128)
    q_host = torch.from_numpy(qh).pin_memory()
    qd = q_host.cuda()
    ids = torch.empty((a.nbatches, B, k), dtype=torch.int32, device="cuda")
    dd = torch.empty((a.nbatches, B, k), dtype=torch.float32, device="cuda")
    qs = torch.empty((a.nbatches, B, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    ids_h = torch.empty((a.nbatches, B, k), dtype=torch.int32).pin_memory()
    dd_h = torch.empty((a.nbatches, B, k), dtype=torch.float32).pin_memory()
    lines = []
    for spec in a.variants.split(","):
        var, S = spec.split(":")
        S = int(S)
        streams = [torch.cuda.Stream() for _ in range(S)]
        qbuf = [torch.empty((B, 128), dtype=torch.float32, device="cuda") for _ in range(S)]

        def step(i):
            b, si = i % a.nbatches, i % S
            st = streams[si]
            with torch.cuda.stream(st):
                src = qd[b * B:(b + 1) * B]
                if var == "zc":
                    idx.knn_device(q_host[b * B:(b + 1) * B].data_ptr(), B, k, ef, ids_h[b].data_ptr(),
                                   dd_h[b].data_ptr(), qs[b].data_ptr(), stream=st.cuda_stream)
                    return
                if var in ("full", "h2d"):
                    qbuf[si].copy_(q_host[b * B:(b + 1) * B], non_blocking=True)
                    src = qbuf[si]
                idx.knn_device(src.data_ptr(), B, k, ef, ids[b].data_ptr(), dd[b].data_ptr(), qs[b].data_ptr(),
                               stream=st.cuda_stream)
                if var in ("full", "d2h"):
                    ids_h[b].copy_(ids[b], non_blocking=True)
                    dd_h[b].copy_(dd[b], non_blocking=True)

        for i in range(2 * S):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        line = {"variant": var, "streams": S, "qps": a.steps * B / el, "ms_per_step": el * 1e3 / a.steps}
        if var in ("zc", "full", "d2h"):  # the host copies hold the answers of the last steps: same as on the device
            last = [(a.steps - 1 - j) % a.nbatches for j in range(min(S, a.nbatches))]
            line["host_results_match_device"] = bool(all(torch.equal(ids_h[b], ids[b].cpu()) for b in last)) \
                if var != "zc" else None
        log(json.dumps(line))
        lines.append(line)
        for s in streams:
            idx.release_stream(s.cuda_stream)
    idx.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(x) + "\n" for x in lines))


if __name__ == "__main__":
    main()
