#!/usr/bin/env python3
"""The low-ef end of the bench's recall / QPS curve (ef = 32 ran no faster than ef = 48): per ef, the fast
kernel's QPS with four batches in flight over K steps, its algorithmic bytes per query and the HBM rate they imply,
and the same with the fallback passes' launches removed (SHINE_DEBUG_MAIN_ONLY, a measurement hook: those launches
have nothing to do at these shapes).  The bench's index (SIFT-shaped 1M x 128, M=16, efC=200, GPU-built).

Usage: python tools/ef_floor.py [--efs 16,24,32,48,64,128] [--steps 200]
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
    p.add_argument("--efs", default="16,24,32,48,64,128")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs", default=";SHINE_DEBUG_MAIN_ONLY=1", help="';'-separated variants (KEY=VALUE[,KEY=VALUE])")
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "ef_floor.jsonl"))
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from config_lines import reserve_streams
    streams = reserve_streams(torch, 4)
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    base = D.sift_like(1_000_000, seed=1)
    B, nb = 1024, 12
    q = D.sift_like(B * nb, seed=2)
    with shine_amd.GpuBuild(base, 16, 200, L.METRIC_L2, seed=1234) as gb:
        idx = gb.open()
    idx.set_search_mode(L.MODE_FAST)
    qd = torch.from_numpy(q).cuda()
    ids = torch.empty((nb, B, 10), dtype=torch.int32, device="cuda")
    qs = torch.zeros((nb, B, L.QS_WORDS), dtype=torch.int32, device="cuda")

    def step(i, ef):
        b = i % nb
        idx.knn_device(qd[b * B:(b + 1) * B].data_ptr(), B, 10, ef, ids[b].data_ptr(), None, qs[b].data_ptr(),
                       stream=streams[i % 4].cuda_stream)

    lines = []
    for env in a.envs.split(";"):
        kv = [x.partition("=") for x in env.split(",") if x]
        for k_, _, v_ in kv:
            os.environ[k_] = v_
        for ef in [int(x) for x in a.efs.split(",")]:
            for i in range(nb + a.warmup):
                step(i, ef)
            torch.cuda.synchronize()
            st = qs.cpu().numpy().view(np.uint32).reshape(-1, L.QS_WORDS)
            bq = idx.algorithmic_bytes(st) / st.shape[0]
            t0 = time.perf_counter()
            for i in range(a.steps):
                step(i, ef)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            qps = a.steps * B / el
            d = {"env": env, "ef": ef, "qps": qps, "ms_per_step": el * 1e3 / a.steps,
                 "bytes_per_query": bq, "gbps": qps * bq / 1e9, "frac": qps * bq / 8e12,
                 "mean_distcomps": float(st[:, 0].mean()), "mean_lists_l0": float(st[:, 4].mean())}
            log(json.dumps(d))
            lines.append(d)
        for k_, _, _ in kv:
            del os.environ[k_]
    idx.close()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "a") as f:
        for d in lines:
            f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
