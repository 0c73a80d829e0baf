#!/usr/bin/env python3
"""Diagnostics (GPU box): one workload of tools/scale_lines.py built once, then measured (config_lines.measure) under
several environment variants of the library's shape hooks, in one process on the same reserved streams.  The variant
list is ';'-separated, each a ','-separated list of NAME=VALUE (an empty variant = the defaults).  The library reads
its hooks on every call, so a variant takes effect at the next search.

Usage: python tools/env_scan.py --which cfg3 --modes exact --envs ";SHINE_EXACT_TWO_CHOICE=1,SHINE_DEBUG_VISCAP=4096"
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
from scale_lines import WORKLOADS, queries  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--which", default="cfg3")
    p.add_argument("--n", type=int, default=0)
    p.add_argument("--envs", default="")
    p.add_argument("--modes", default="exact")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--nbatches", type=int, default=10)
    p.add_argument("--inflight", type=int, default=4)
    p.add_argument("--ef", default="")
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "env_scan.jsonl"))
    a = p.parse_args()
    import torch
    import shine_amd
    from shine_amd import datasets as D
    torch.cuda.set_device(0)
    reserve_streams(torch, a.inflight)
    kind, n, dim, metric, elem, M, efc, ef, batch, alpha = WORKLOADS[a.which]
    n = a.n or n
    base = D.generate_device(kind, n, seed=1, d=dim)
    q = queries(torch, D, kind, dim, batch * a.nbatches, alpha)
    with Heartbeat("gt"):
        gt = D.ground_truth_device(base, q, a.k, metric)
    with Heartbeat("build"):
        gb = shine_amd.GpuBuild(base.data_ptr(), M, efc, metric, seed=1234, n=n, dim=dim)
    del base
    torch.cuda.empty_cache()
    idx = gb.open(elem)
    gb.close()
    a.ef = a.ef or str(ef)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    for env in a.envs.split(";"):
        kv = [x.partition("=") for x in env.split(",") if x]
        for k_, _, v_ in kv:
            os.environ[k_] = v_
        for line in measure(torch, idx, a.which, a, q, gt, batch, 1, ef):
            line["env"] = env
            log(json.dumps({k: line[k] for k in ("env", "search_mode", "value", "recall_at_10")}))
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")
        for k_, _, _ in kv:
            del os.environ[k_]
    idx.close()


if __name__ == "__main__":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # batches in flight on distinct hardware queues (the box exports 4)
    main()
