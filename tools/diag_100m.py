#!/usr/bin/env python3
"""Diagnostics (GPU box): the DEEP-shaped 100M-record index (GPU-built), QPS with four batches in flight per search
mode and ef under environment variants (visited-table policy hooks), and recall against float64 ground truth.

Usage: python tools/diag_100m.py [--n 100000000] [--runs fast:128,exact:128] [--envs ";SHINE_DEBUG_NO_SPILL=1"]
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
from config_lines import Heartbeat  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100_000_000)
    p.add_argument("--kind", default="deep_like")
    p.add_argument("--dim", type=int, default=96)
    p.add_argument("--metric", type=int, default=0)
    p.add_argument("--runs", default="fast:64,fast:128,fast:256,exact:128")
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--envs", default=";SHINE_DEBUG_NO_SPILL=1;SHINE_DEBUG_VISCAP=8192")
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from config_lines import reserve_streams
    all_streams = reserve_streams(torch, 8)  # first streams of the process: distinct hardware queues
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    base = D.generate_device(a.kind, a.n, seed=1, d=a.dim)
    q = D.generate_device(a.kind, 8192, seed=2, d=a.dim)
    with Heartbeat("gt"):
        gt = D.ground_truth_device(base, q, 10, a.metric)
    t0 = time.time()
    with Heartbeat("build"):
        gb = shine_amd.GpuBuild(base.data_ptr(), 16, 200, a.metric, seed=1234, n=a.n, dim=a.dim)
    log(f"built in {time.time() - t0:.1f}s: {json.dumps(gb.stats())}")
    del base
    torch.cuda.empty_cache()
    idx = gb.open()
    qh = q.cpu().numpy()
    B, nb = 1024, 8
    ids = torch.empty((nb, B, 10), dtype=torch.int32, device="cuda")
    qs = torch.zeros((nb, B, L.QS_WORDS), dtype=torch.int32, device="cuda")
    streams = all_streams[:4]

    def run(steps, ef):
        for i in range(steps):
            b = i % nb
            idx.knn_device(q[b * B:(b + 1) * B].data_ptr(), B, 10, ef, ids[b].data_ptr(), None, qs[b].data_ptr(),
                           stream=streams[i % len(streams)].cuda_stream)

    for env in a.envs.split(";"):
        for kv in env.split(","):
            k_, _, v_ = kv.partition("=")
            if k_:
                os.environ[k_] = v_
        for spec in a.runs.split(","):
            mode_name, ef, *inf = spec.split(":")
            ef = int(ef)
            streams = all_streams[:int(inf[0]) if inf else 4]
            idx.set_search_mode(L.MODE_FAST if mode_name == "fast" else L.MODE_EXACT)
            run(2 * nb, ef)
            torch.cuda.synchronize()
            st = qs.cpu().numpy().view(np.uint32).reshape(-1, L.QS_WORDS)
            rec = D.recall_at_k(ids.cpu().numpy().view(np.uint32).reshape(-1, 10), gt[:nb * B], 10)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(a.steps, ef)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            vis = st[:, 1].astype(np.int64) + st[:, 2]
            log(json.dumps({"env": env, "mode": mode_name, "ef": ef, "inflight": len(streams), "qps": a.steps * B / el,
                            "recall": rec,
                            "failed": int((st[:, 6] != 0).sum()), "visited_mean": float(vis.mean()),
                            "visited_p99": float(np.percentile(vis, 99)), "visited_max": int(vis.max()),
                            "distcomps": float(st[:, 0].mean())}))
        for kv in env.split(","):
            k_, _, _ = kv.partition("=")
            if k_:
                del os.environ[k_]
    idx.close()
    gb.close()


if __name__ == "__main__":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # batches in flight on distinct hardware queues (the box exports 4)
    main()
