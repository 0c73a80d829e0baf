#!/usr/bin/env python3
"""One library build, one process (diagnostics): QPS of the bench's workload per search mode and ef, four batches in
flight on four hardware queues, 100 steps after a warmup.  Run it once per build, alternating builds on one box:
two builds in one process (tools/ab_lib.py) share the process's hardware queues, and with four streams per side the
second side's streams collide on them (it measured up to 28 % slower whichever build it was, profiles/r02/
ab_order_bias.txt).

Usage: SHINE_GPU_LIB=_abl/libX.so python tools/lib_probe.py --runs fast:48,fast:128,exact:128,fast:128:u8 --tag X
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
    p.add_argument("--runs", default="fast:48,fast:128,exact:128")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--tag", default=os.environ.get("SHINE_GPU_LIB", "in-tree"))
    p.add_argument("--cache", default=os.environ.get("SHINE_BENCH_CACHE", "/tmp/shine_bench"))
    a = p.parse_args()
    import numpy as np
    import torch
    import shine_amd
    from shine_amd import datasets as D
    from bench import host_threads, prepare_dumps

    B, nb, S = 1024, 12, 4
    key = hashlib.sha1(f"{1_000_000}-128-16-200-1-sift_like-v3".encode()).hexdigest()[:12]
    paths = [Path(a.cache) / key / "dump" / shine_amd.dump_name(16, 200, 0, 1)]

    def build():
        return shine_amd.build(D.sift_like(1_000_000, seed=1, d=128), 16, 200, 0, 1, seed=1234,
                               threads=host_threads())[0]

    prepare_dumps(paths, 0, None, build)
    opened = {}

    def index(rows):  # f32 rows (the bench's `value`) or u8 rows (lossless for SIFT-shaped records)
        if rows not in opened:
            elem = shine_amd.ELEM_U8 if rows == "u8" else shine_amd.ELEM_F32
            opened[rows] = shine_amd.Index.open(paths, 128, 16, shine_amd.METRIC_L2, elem=elem, gpus=[0])
        return opened[rows]
    q = torch.from_numpy(D.sift_like(B * nb, seed=2, d=128)).cuda()
    ids = torch.empty((nb, B, 10), dtype=torch.int32, device="cuda")
    qs = torch.empty((nb, B, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(S)]

    def run(steps, ef):
        idx = cur[0]
        for i in range(steps):
            b = i % nb
            idx.knn_device(q[b * B:(b + 1) * B].data_ptr(), B, 10, ef, ids[b].data_ptr(), None, qs[b].data_ptr(),
                           stream=streams[i % S].cuda_stream)

    cur = [None]
    for spec in a.runs.split(","):
        mode, ef, *rows = spec.split(":")
        ef = int(ef)
        rows = rows[0] if rows else "f32"
        idx = cur[0] = index(rows)
        idx.set_search_mode(shine_amd.MODE_FAST if mode == "fast" else shine_amd.MODE_EXACT)
        run(2 * nb, ef)
        torch.cuda.synchronize()
        st = qs.cpu().numpy().view(np.uint32).reshape(-1, shine_amd.QS_WORDS)
        assert (st[:, 6] == 0).all()
        t0 = time.perf_counter()
        run(a.steps, ef)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"tag": a.tag, "mode": mode, "ef": ef, "rows": rows, "qps": a.steps * B / el}), flush=True)
    for idx in opened.values():
        idx.close()


if __name__ == "__main__":
    main()
