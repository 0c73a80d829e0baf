#!/usr/bin/env python3
"""Host-API rate of the drop-in path (shine_knn_batch) on the bench's index (SIFT-shaped 1M x 128, M=16, efC=200,
GPU-built, ef=128, fast mode), against the HBM-resident rate with four batches in flight:
  * one call per 1,024-query batch (the round-4 bench leg: nothing in flight between calls);
  * one call over the whole query set (12,288 or --nq), split inside the library into SHINE_HOST_CHUNK-query chunks
    kept in flight on the slot's host streams (capi.cc knn_host), for several chunk sizes (0 = one launch).
Every variant's ids are checked against the one-launch call.  One JSON line per variant.

Usage: python tools/host_api_probe.py [--nq 12288] [--chunks 0,512,1024,2048,4096] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
from bench import log  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--nq", type=int, default=12288)
    p.add_argument("--ef", type=int, default=128)
    p.add_argument("--chunks", default="0,512,1024,2048,4096")
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "host_api_probe.jsonl"))
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from config_lines import reserve_streams
    streams = reserve_streams(torch, 4)
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    base = D.sift_like(a.n, seed=1)
    q = D.sift_like(a.nq, seed=2)
    with shine_amd.GpuBuild(base, 16, 200, L.METRIC_L2, seed=1234) as gb:
        idx = gb.open()
    idx.set_search_mode(L.MODE_FAST)
    lines = []

    def emit(d):
        log(json.dumps(d))
        lines.append(d)

    os.environ["SHINE_HOST_CHUNK"] = "0"
    want = idx.knn(q, 10, a.ef).ids
    # HBM-resident, four batches in flight (the bench's `value`)
    B = 1024
    nb = a.nq // B
    qd = torch.from_numpy(q).cuda()
    ids = torch.empty((nb, B, 10), dtype=torch.int32, device="cuda")

    def dev_step(i):
        b = i % nb
        idx.knn_device(qd[b * B:(b + 1) * B].data_ptr(), B, 10, a.ef, ids[b].data_ptr(), None, None,
                       stream=streams[i % 4].cuda_stream)

    for i in range(2 * nb):
        dev_step(i)
    torch.cuda.synchronize()
    steps = nb * a.reps
    t0 = time.perf_counter()
    for i in range(steps):
        dev_step(i)
    torch.cuda.synchronize()
    dev_qps = steps * B / (time.perf_counter() - t0)
    emit({"variant": "device_4_in_flight", "qps": dev_qps})
    # one host call per batch
    for i in range(nb):
        idx.knn(q[i * B:(i + 1) * B], 10, a.ef)
    t0 = time.perf_counter()
    for r in range(a.reps):
        for i in range(nb):
            idx.knn(q[i * B:(i + 1) * B], 10, a.ef)
    qps = a.reps * nb * B / (time.perf_counter() - t0)
    emit({"variant": "host_call_per_batch", "qps": qps, "vs_device": qps / dev_qps})
    for ch in [int(x) for x in a.chunks.split(",")]:
        os.environ["SHINE_HOST_CHUNK"] = str(ch)
        r = idx.knn(q, 10, a.ef)
        same = bool((r.ids == want).all())
        t0 = time.perf_counter()
        for _ in range(a.reps):
            idx.knn(q, 10, a.ef)
        qps = a.reps * a.nq / (time.perf_counter() - t0)
        emit({"variant": "host_call_whole_set", "chunk": ch, "nq": a.nq, "qps": qps, "vs_device": qps / dev_qps,
              "same_ids_as_one_launch": same, "kernel_ms": r.stats["kernel_ms"]})
    idx.close()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "a") as f:
        for d in lines:
            f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
