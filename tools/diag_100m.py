#!/usr/bin/env python3
"""Diagnostics (GPU box): the DEEP-shaped 100M-record index (GPU-built), fast / exact search shapes and timings per ef
through the host API (kernel time, hand-ons), with the spill on and off, and recall against ground truth.

Usage: python tools/diag_100m.py [--n 100000000] [--efs 64,128,256]
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
    p.add_argument("--efs", default="64,128,256")
    p.add_argument("--calls", type=int, default=4)
    p.add_argument("--envs", default=",SHINE_DEBUG_NO_SPILL=1")
    a = p.parse_args()
    import torch
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    base = D.generate_device(a.kind, a.n, seed=1, d=a.dim)
    q = D.generate_device(a.kind, 4096, seed=2, d=a.dim)
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
    os.environ["SHINE_DEBUG_SHAPE"] = "1"
    for env in a.envs.split(","):
        k_, _, v_ = env.partition("=")
        if k_:
            os.environ[k_] = v_
        for mode_name, mode in (("fast", L.MODE_FAST), ("exact", L.MODE_EXACT)):
            idx.set_search_mode(mode)
            for ef in [int(x) for x in a.efs.split(",")]:
                rows = []
                for c in range(a.calls):
                    b = c % 4
                    r = idx.knn(qh[b * 1024:(b + 1) * 1024], 10, ef)
                    rows.append((r.stats["kernel_ms"], r.stats["overflow_retries"]))
                rec = D.recall_at_k(r.ids, gt[(b * 1024):(b + 1) * 1024], 10)
                vis = r.qstats[:, 1].astype(np.int64) + r.qstats[:, 2]
                log(json.dumps({"env": env, "mode": mode_name, "ef": ef, "kernel_ms": [x[0] for x in rows],
                                "handed_on": [x[1] for x in rows], "recall": rec,
                                "visited_mean": float(vis.mean()), "visited_p99": float(np.percentile(vis, 99)),
                                "visited_max": int(vis.max()), "distcomps": float(r.qstats[:, 0].mean())}))
        if k_:
            del os.environ[k_]
    idx.close()
    gb.close()


if __name__ == "__main__":
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    main()
