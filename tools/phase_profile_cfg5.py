#!/usr/bin/env python3
"""Diagnostics (GPU box): per-phase shader-clock shares of search_fast_kernel<200, IP, __half, R=4> — cfg5's shape
(TTI-shaped rows, fp16 records, inner product, ef = 250) — on a GPU-built index of --n records (default 10M).

Runs one 1,024-query batch of the Zipf(1.0) mix plain, then the PROF variant (SHINE_PHASE_PROFILE=1: s_memtime stamps,
its run time is not quoted); the library prints the cycle totals per phase (capi.cc print_phase_profile) to stderr.

Usage: python tools/phase_profile_cfg5.py [--n 10000000] [--ef 250]
"""
from __future__ import annotations

import argparse
import os
import sys
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
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--ef", type=int, default=250)
    p.add_argument("--rows", default="f16", choices=["f16", "f32"])
    a = p.parse_args()
    import torch
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    base = D.generate_device("tti_like", a.n, seed=1, d=200)
    with Heartbeat("GPU build"):
        gb = shine_amd.GpuBuild(base.data_ptr(), 16, 200, 1, seed=1234, n=a.n, dim=200)
    del base
    torch.cuda.empty_cache()
    idx = gb.open(L.ELEM_F16 if a.rows == "f16" else L.ELEM_F32)
    gb.close()
    idx.set_search_mode(L.MODE_FAST)
    pool = D.generate_device("tti_like", 500_000, seed=2, d=200).cpu().numpy()
    q, _, _ = D.zipf_query_mix(pool, 4096, 1.0, seed=3)
    q = np.ascontiguousarray(q)
    for i in range(3):  # learn the table shape from a few calls first, as the timed runs do
        r = idx.knn(q[1024 * i:1024 * (i + 1)], 10, a.ef)
    qb = q[3072:]
    r = idx.knn(qb, 10, a.ef)
    log(f"plain kernel_ms {r.stats['kernel_ms']:.3f} mean distcomps {r.qstats[:, 0].mean():.1f} "
        f"mean L0 lists {r.qstats[:, 4].mean():.1f}")
    os.environ["SHINE_DEBUG_SHAPE"] = "1"
    os.environ["SHINE_PHASE_PROFILE"] = "1"
    r = idx.knn(qb, 10, a.ef)
    log(f"profiled kernel_ms {r.stats['kernel_ms']:.3f}")
    idx.close()


if __name__ == "__main__":
    main()
