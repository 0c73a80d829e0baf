#!/usr/bin/env python3
"""Queries in flight x visited-table size x row storage (diagnostics, fast mode, bench index).

For every setting: QPS over --steps batches with --inflight batches on as many streams, and the share of queries the
main pass handed on to the light pass (shine_knn_batch's overflow_retries over one batch).  Settings are
'rows:inflight:viscap[:load]' (viscap 0 = the library's own choice; load: SHINE_DEBUG_VISLOAD), e.g. --settings f32:2:0,u8:3:4096.
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
    p.add_argument("--settings", required=True)
    p.add_argument("--ef", type=int, default=128)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--nbatches", type=int, default=12)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--out", default="")
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
    qh = D.sift_like(a.batch * a.nbatches, seed=2, d=128)
    q = torch.from_numpy(qh).cuda()
    ids = torch.empty((a.nbatches, a.batch, 10), dtype=torch.int32, device="cuda")
    qs = torch.zeros((a.nbatches, a.batch, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    idx = {}
    lines = []
    for spec in a.settings.split(","):
        rows, inflight, viscap, *rest = spec.split(":")
        inflight, viscap = int(inflight), int(viscap)
        if rest:
            os.environ["SHINE_DEBUG_VISLOAD"] = rest[0]
        else:
            os.environ.pop("SHINE_DEBUG_VISLOAD", None)
        if rows not in idx:
            elem = shine_amd.ELEM_U8 if rows == "u8" else shine_amd.ELEM_F32
            idx[rows] = shine_amd.Index.open(paths, 128, 16, shine_amd.METRIC_L2, elem=elem, gpus=[0])
            idx[rows].set_search_mode(shine_amd.MODE_FAST)
        ix = idx[rows]
        if viscap:
            os.environ["SHINE_DEBUG_VISCAP"] = str(viscap)
        else:
            os.environ.pop("SHINE_DEBUG_VISCAP", None)
        streams = [torch.cuda.Stream() for _ in range(inflight)]

        def step(i):
            b = i % a.nbatches
            s = streams[i % inflight]
            ix.knn_device(q[b * a.batch:(b + 1) * a.batch].data_ptr(), a.batch, 10, a.ef, ids[b].data_ptr(), None,
                          qs[b].data_ptr(), stream=s.cuda_stream)

        for i in range(2 * a.nbatches):
            step(i)
        torch.cuda.synchronize()
        st = qs.cpu().numpy().view(np.uint32).reshape(-1, shine_amd.QS_WORDS)
        if (st[:, 6] != 0).any():
            raise SystemExit(f"{spec}: queries failed")
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        r = ix.knn(qh[:a.batch], 10, a.ef)
        line = {"setting": spec, "ef": a.ef, "qps": a.steps * a.batch / el, "ms_per_batch": el * 1e3 / a.steps,
                "handed_on_share": r.stats["overflow_retries"] / a.batch,
                "visited_p99": float(np.percentile(st[:, 1] + st[:, 2], 99))}
        log(json.dumps(line))
        lines.append(line)
        for s in streams:
            ix.release_stream(s.cuda_stream)
    for ix in idx.values():
        ix.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(x) + "\n" for x in lines))


if __name__ == "__main__":
    main()
