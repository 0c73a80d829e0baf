#!/usr/bin/env python3
"""Interleaved A/B timing of two builds of libshine_gpu.so in ONE process (diagnostics).

Caution (round 2): with four streams per side the second side's streams collide on the process's hardware queues and
it measures up to 28 % slower whichever build it is (profiles/r02/ab_order_bias.txt); compare builds one process
each with tools/lib_probe.py instead, alternating builds on one box.

Each library opens the bench's dump by itself (shine_open, fast mode) and answers the same query batches on its own
pair of HIP streams; timed blocks alternate A, B, A, B, ... so box and clock drift hit both equally.  Only the
entry points whose signatures are unchanged since round 1 are used (shine_open, shine_set_search_mode,
shine_knn_batch_device, shine_close), so an older build can be the A side.

Usage: GPU_MAX_HW_QUEUES=16 python tools/ab_lib.py --libs _abl/libshine_r01.so,dm-hnsw-reference_amd/libshine_gpu.so --ef 32,128
(with the default 4 hardware queues the streams of several sides share queues and one side can lose its overlap)
Per-library environment (the SHINE_DEBUG_* hooks) goes after '@': --libs "a.so,b.so@SHINE_DEBUG_NO_SEEN=1".
"""
from __future__ import annotations

import argparse
import ctypes as C
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
    p.add_argument("--libs", required=True, help="','-separated library paths, each optionally '@VAR=V;VAR=V'")
    p.add_argument("--ef", default="32,128")
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--nbatches", type=int, default=10)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--inflight", type=int, default=2)
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--mode", default="fast", choices=["fast", "exact"])
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
    q = torch.from_numpy(D.sift_like(a.batch * a.nbatches, seed=2, d=128)).cuda()
    sides = []
    for spec in a.libs.split(","):
        path, _, env = spec.partition("@")
        lib = C.CDLL(str(ROOT / path) if not os.path.isabs(path) else path)
        lib.shine_last_error.restype = C.c_char_p
        h = C.c_void_p()
        cp = (C.c_char_p * 1)(str(paths[0]).encode())
        gpu = (C.c_int * 1)(0)
        if lib.shine_open(cp, 1, 128, 16, shine_amd.METRIC_L2, 0, gpu, 1, C.byref(h)) != 0:
            raise SystemExit(f"{path}: {lib.shine_last_error()}")
        if lib.shine_set_search_mode(h, shine_amd.MODE_FAST if a.mode == "fast" else shine_amd.MODE_EXACT) != 0:
            raise SystemExit(f"{path}: {lib.shine_last_error()}")
        envd = dict(kv.split("=", 1) for kv in env.split(";") if kv)
        ids = torch.empty((a.nbatches, a.batch, 10), dtype=torch.int32, device="cuda")
        qs = torch.zeros((a.nbatches, a.batch, 16), dtype=torch.int32, device="cuda")
        streams = [torch.cuda.Stream() for _ in range(a.inflight)]
        sides.append((spec, lib, h, envd, ids, qs, streams))

    def run(side, ef, steps):
        _, lib, h, _, ids, qs, streams = side
        for i in range(steps):
            b = i % a.nbatches
            rc = lib.shine_knn_batch_device(h, 0, C.c_void_p(q[b * a.batch:(b + 1) * a.batch].data_ptr()), a.batch,
                                            10, ef, C.c_void_p(ids[b].data_ptr()), None,
                                            C.c_void_p(qs[b].data_ptr()), C.c_void_p(streams[i % len(streams)].cuda_stream))
            if rc != 0:
                raise SystemExit(f"{side[0]}: {lib.shine_last_error()}")

    results = {}
    for ef in [int(x) for x in a.ef.split(",")]:
        for rep in range(a.reps):
            for si, side in enumerate(sides):
                saved = {k: os.environ.get(k) for k in side[3]}
                os.environ.update(side[3])
                run(side, ef, a.nbatches)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(side, ef, a.steps)
                torch.cuda.synchronize()
                results.setdefault((si, ef), []).append(a.steps * a.batch / (time.perf_counter() - t0))
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        ref = sides[0][4].cpu().numpy()
        for side in sides[1:]:
            same = float((np.sort(side[4].cpu().numpy(), -1) == np.sort(ref, -1)).all(-1).mean())
            line = {"ef": ef, "lib": side[0], "same_id_sets_as_first": same}
            print(json.dumps(line), flush=True)
    for (si, ef), v in sorted(results.items(), key=lambda x: (x[0][1], x[0][0])):
        line = {"lib": sides[si][0], "ef": ef, "qps_median": float(np.median(v)), "qps": [round(x) for x in v]}
        print(json.dumps(line), flush=True)
        log(json.dumps(line))
    for side in sides:
        side[1].shine_close(side[2])


if __name__ == "__main__":
    main()
