#!/usr/bin/env python3
"""Diagnostics (GPU box): one GPU-built DEEP-shaped index (default 10M x 96, L2, ef 128) opened in several layouts on
one GPU — replica (hipMalloc arrays), sharded over 1 slot (VM-mapped stripe views, read accounting on), sharded over 8
slots — and measured alike (tools/config_lines.measure, four batches in flight on reserved streams), to separate the
sharded layout's own cost from the slot emulation's.  Usage: python tools/layout_probe.py [--n 10000000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
from bench import log  # noqa: E402
from config_lines import Heartbeat, measure, reserve_streams  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--layouts", default="replica:1,sharded:1,sharded:8")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--nbatches", type=int, default=8)
    p.add_argument("--inflight", type=int, default=4)
    p.add_argument("--ef", default="128")
    p.add_argument("--modes", default="fast")
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "layout_probe.jsonl"))
    a = p.parse_args()
    import torch
    import shine_amd
    from shine_amd import datasets as D
    torch.cuda.set_device(0)
    reserve_streams(torch, a.inflight * 8)
    base = D.generate_device("deep_like", a.n, seed=1, d=96)
    batch = 1024
    q = D.generate_device("deep_like", batch * a.nbatches, seed=2, d=96)
    with Heartbeat("gt"):
        gt = D.ground_truth_device(base, q, a.k, 0)
    with Heartbeat("build"):
        gb = shine_amd.GpuBuild(base.data_ptr(), 16, 200, 0, seed=1234, n=a.n, dim=96)
    del base
    torch.cuda.empty_cache()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    for spec in a.layouts.split(","):
        placement, slots = spec.split(":")
        slots = int(slots)
        idx = gb.open_ex(8 if placement == "sharded" else 1, gpus=[0] * slots, placement=placement)
        for line in measure(torch, idx, f"layout-{placement}-{slots}", a, q, gt, batch * slots // slots, slots, 128):
            line["layout"] = {"placement": placement, "slots": slots}
            log(json.dumps(line))
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")
        idx.close()
    gb.close()


if __name__ == "__main__":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # batches in flight on distinct hardware queues (the box exports 4)
    main()
