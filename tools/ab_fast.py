#!/usr/bin/env python3
"""Interleaved A/B timing of search configurations in ONE process on the bench's index (diagnostics).

The C ABI reads its SHINE_DEBUG_* launch hooks at every call, so configurations are switched through os.environ
between timed blocks: A, B, A, B, ... with the same index, queries, streams and warm caches, which removes the
box-to-box and run-to-run noise that separate bench.py runs carry.  Prints one JSON line per (config, ef) with the
median QPS over --reps blocks.

Usage: python tools/ab_fast.py --configs "SHINE_DEBUG_VIS16=1;SHINE_DEBUG_VIS16=0" --ef 32,128 [--inflight 2]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", required=True, help="';'-separated configs, each a ','-separated list of VAR=VALUE")
    p.add_argument("--ef", default="128")
    p.add_argument("--mode", default="fast")
    p.add_argument("--inflight", type=int, default=2)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--nbatches", type=int, default=10)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--cache", default=os.environ.get("SHINE_BENCH_CACHE", "/tmp/shine_bench"))
    a = p.parse_args()
    import torch
    import shine_amd
    from shine_amd import datasets as D
    from bench import host_threads, log, prepare_dumps

    key = hashlib.sha1(f"{a.n}-128-16-200-1-sift_like-v3".encode()).hexdigest()[:12]
    paths = [Path(a.cache) / key / "dump" / shine_amd.dump_name(16, 200, 0, 1)]

    def build():
        base = D.sift_like(a.n, seed=1, d=128)
        dumps, _ = shine_amd.build(base, 16, 200, shine_amd.METRIC_L2, 1, seed=1234, threads=host_threads())
        return dumps

    prepare_dumps(paths, 0, None, build)
    idx = shine_amd.Index.open(paths, 128, 16, shine_amd.METRIC_L2, gpus=[0])
    idx.set_search_mode(shine_amd.MODE_FAST if a.mode == "fast" else shine_amd.MODE_EXACT)
    q = torch.from_numpy(D.sift_like(a.batch * a.nbatches, seed=2, d=128)).cuda()
    ids = torch.empty((a.nbatches, a.batch, 10), dtype=torch.int32, device="cuda")
    qs = torch.zeros((a.nbatches, a.batch, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(a.inflight)]
    configs = [dict(kv.split("=", 1) for kv in c.split(",") if kv) for c in a.configs.split(";")]

    def run(ef, steps):
        for i in range(steps):
            b = i % a.nbatches
            idx.knn_device(q[b * a.batch:(b + 1) * a.batch].data_ptr(), a.batch, 10, ef, ids[b].data_ptr(), None,
                           qs[b].data_ptr(), stream=streams[i % len(streams)].cuda_stream)

    results = {}
    for ef in [int(x) for x in a.ef.split(",")]:
        for rep in range(a.reps):
            for ci, cfg in enumerate(configs):
                saved = {k: os.environ.get(k) for k in cfg}
                os.environ.update(cfg)
                run(ef, a.nbatches)  # warm: one pass over every batch with this config
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(ef, a.steps)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                st = qs.cpu().numpy().view(np.uint32).reshape(-1, shine_amd.QS_WORDS)
                if (st[:, 6] != 0).any():
                    raise SystemExit(f"config {cfg}: failed queries")
                results.setdefault((ci, ef), []).append(a.steps * a.batch / el)
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    for (ci, ef), v in sorted(results.items(), key=lambda x: (x[0][1], x[0][0])):
        line = {"config": a.configs.split(";")[ci], "ef": ef, "qps_median": float(np.median(v)),
                "qps": [round(x) for x in v]}
        print(json.dumps(line), flush=True)
        log(json.dumps(line))
    idx.close()


if __name__ == "__main__":
    main()
