#!/usr/bin/env python3
"""The drop-in façade end to end: shine_compute_node — the reference's ComputeNode driver rebuilt on the
C ABI — over big-ann files of the bench's workload (SIFT-shaped 1M x 128 as base.u8bin, 10,000 queries as
queries/query-sift.u8bin, float64 ground truth as groundtruth-sift.bin), with the reference's flags:
  1. --store-index --builder gpu: build on the GPU (shine_gpu_build), store the memory-node dumps, run the queries;
  2. --load-index: reopen the stored dumps and run the queries again (the reference's usual split of the two runs).
Both runs pass the whole query set to shine_knn_batch in one call (--batch 0, the library keeps 1,024-query chunks in
flight).  Prints each run's statistics JSON (queries.queries_per_sec, queries.recall, timings) as one line.

Usage: python tools/compute_node_run.py [--n 1000000] [--nq 10000] [--ef 128] [--mode fast] [--dir /tmp/cn]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT))
from bench import ground_truth, log  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--nq", type=int, default=10_000)
    p.add_argument("--ef", type=int, default=128)
    p.add_argument("--mode", default="fast")
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--dir", default="/tmp/shine_cn")
    p.add_argument("--inflight", default="2,3", help="--load-index runs with these --calls-in-flight as well")
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "compute_node_run.jsonl"))
    a = p.parse_args()
    import torch
    from shine_amd import datasets as D
    from shine_amd import formats as F
    d = Path(a.dir)
    (d / "queries").mkdir(parents=True, exist_ok=True)
    t0 = time.time()
    base = D.sift_like(a.n, seed=1)
    q = D.sift_like(a.nq, seed=2)
    F.write_vectors(d / "base.u8bin", base)
    F.write_vectors(d / "queries" / "query-sift.u8bin", q)
    gt = ground_truth(torch, base, q, 100, 0).astype("uint32")
    F.write_vectors(d / "queries" / "groundtruth-sift.bin", gt)
    del base
    torch.cuda.empty_cache()
    log(f"files written in {time.time() - t0:.1f}s")
    exe = ROOT / "dm-hnsw-reference_amd" / "shine_compute_node"
    common = ["-d", str(d), "-q", "sift", "-t", str(a.threads), "--ef-search", str(a.ef), "-k", "10", "-m", "16",
              "--ef-construction", "200", "--search-mode", a.mode]
    lines = []
    runs = [("store_gpu_build", ["--store-index", "--builder", "gpu"]), ("load", ["--load-index"])]
    for n in (int(x) for x in a.inflight.split(",") if x.strip()):  # host calls kept in flight (shine_knn_batch_async)
        runs.append((f"load_inflight{n}", ["--load-index", "--calls-in-flight", str(n)]))
    for label, extra in runs:
        t1 = time.time()
        r = subprocess.run([str(exe), *common, *extra], capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            raise SystemExit(f"{label}: shine_compute_node exited {r.returncode}: {r.stderr[-2000:]}")
        st = json.loads(r.stdout)
        line = {"run": label, "wall_s": time.time() - t1, "args": common + extra, "statistics": st}
        log(f"{label}: {st['queries']['queries_per_sec']} queries/s, recall {st['queries']['recall']}, "
            f"timings {st['timings']}")
        lines.append(line)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "a") as f:
        for line in lines:
            f.write(json.dumps(line) + "\n")
    print(json.dumps(lines))


if __name__ == "__main__":
    main()
