#!/usr/bin/env python3
"""The reference's cache-size-and-skew experiment (scripts/exp_cache_size_and_skew.py:6-13) on the GPU node.

Labels (scripts/config.py get_cache_parameters):
  baseline            no cache                                    -> SHINE_PLACE_SHARDED, no cache
  +cache              --cache --cache-ratio R                     -> SHARDED + SHINE_CACHE_DYNAMIC at R %
  +adaptive-routing   --cache --cache-ratio R --routing           -> SHARDED_REGIONS (query router) + DYNAMIC at R %
Grid: Zipf alpha in {0, 0.5, 0.75, 1.0, 1.25, 1.5} x cache ratio in {2, 4, 5, 6, 8, 10} % (the reference runs every
ratio only at alpha 0 and 1.0 and ratio 5 elsewhere; this replays the full cross), baseline once per alpha.

Workload: the TTI-shaped index (200-d, inner product, fp16 rows) of --n records built on the GPU, laid out over --slots
GPU slots as 8 memory-node dumps (on a one-GPU box the slots repeat device 0: every stripe is its own allocation, so
the read classes — own stripe / cached copy / xGMI — are exact, but every read is local HBM).  Queries: skew.py's
replay of a 500K pool with a warmup split: per cell, --warm calls warm the cache, then --calls calls are
measured (hit rate, recall, host-API QPS including the cache updates between calls).

Usage: python tools/skew_grid.py [--n 10000000] [--slots 8]
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
from config_lines import Heartbeat, read_classes  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--slots", type=int, default=8)
    p.add_argument("--alphas", default="0,0.5,0.75,1.0,1.25,1.5")
    p.add_argument("--ratios", default="2,4,5,6,8,10")
    p.add_argument("--labels", default="baseline,+cache,+adaptive-routing")
    p.add_argument("--warm", type=int, default=24)
    p.add_argument("--calls", type=int, default=8)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--ef", type=int, default=250)
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "skew_grid.jsonl"))
    a = p.parse_args()
    import torch
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    kind, dim, metric, M, efc, k = "tti_like", 200, 1, 16, 200, 10
    ndev = torch.cuda.device_count()
    gpus = [s % ndev for s in range(a.slots)]
    base = D.generate_device(kind, a.n, seed=1, d=dim)
    pool_n = 500_000  # skew.py's query pool (create_queries.py: 500k slice)
    per_cell = (a.warm + a.calls) * a.batch
    pool = D.generate_device(kind, pool_n, seed=2, d=dim)
    with Heartbeat("ground truth"):  # every mix draws from the pool's first per_cell entries (zipf_counts)
        gt_pool = D.ground_truth_device(base, pool[:per_cell], k, metric)
    pool_h = pool.cpu().numpy()
    del pool
    t0 = time.time()
    with Heartbeat("GPU build"):
        gb = shine_amd.GpuBuild(base.data_ptr(), M, efc, metric, seed=1234, n=a.n, dim=dim)
    log(f"built {a.n} x {dim} in {time.time() - t0:.1f}s")
    del base
    torch.cuda.empty_cache()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    opened = {}

    def handle(placement):
        if placement not in opened:
            t1 = time.time()
            with Heartbeat(f"layout {placement}"):
                opened[placement] = gb.open_ex(8, elem=L.ELEM_F16, gpus=gpus, placement=placement)
            opened[placement].set_search_mode(L.MODE_FAST)
            log(f"{placement} layout over {a.slots} slots in {time.time() - t1:.1f}s")
        return opened[placement]

    for label in a.labels.split(","):
        placement = "regions" if "routing" in label else "sharded"
        idx = handle(placement)
        ratios = [None] if label == "baseline" else [float(x) for x in a.ratios.split(",")]
        for alpha in [float(x) for x in a.alphas.split(",")]:
            q, _, src = D.zipf_query_mix(pool_h, per_cell, alpha, seed=13)
            q = np.ascontiguousarray(q)
            for ratio in ratios:
                if ratio is None:
                    idx.set_cache_policy(L.CACHE_STATIC)
                else:
                    idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=ratio, seed=1)
                hits = reads = 0
                res, t_meas, adm, qss, t_warm, kms = [], 0.0, 0, [], 0.0, 0.0
                # the measured calls' clock runs from the first one's start to the end of the last replay they started
                # (the pipelined policy's replay runs past a call's return: shine_cache_wait), the loop's own time in
                # between included
                t_start = None
                for c in range(a.warm + a.calls):
                    qq = q[c * a.batch:(c + 1) * a.batch]
                    t1 = time.perf_counter()
                    if c == a.warm:
                        t_start = t1
                    r = idx.knn(qq, k, a.ef, query_ids=np.arange(c * a.batch, (c + 1) * a.batch, dtype=np.uint32))
                    el = time.perf_counter() - t1
                    if c < a.warm:
                        t_warm += el
                    else:
                        qss.append(r.qstats)
                        hits += r.stats["node_cache_hits"]
                        reads += r.stats["node_reads"]
                        res.append(r.ids)
                        adm += r.stats["cache_admitted"]
                        kms += r.stats["kernel_ms"]
                if ratio is not None:
                    idx.cache_wait()
                t_meas = time.perf_counter() - t_start
                got = np.concatenate(res)
                want = gt_pool[src[a.warm * a.batch:per_cell]]
                line = {"workload": "cfg5-skew-grid", "label": label, "alpha": alpha, "cache_ratio_percent": ratio,
                        "placement": placement, "gpu_slots": a.slots, "physical_gpus": len(set(gpus)),
                        "cache_hit_rate": hits / max(1, reads), "node_reads": reads,
                        "read_classes": read_classes(np.concatenate(qss)),
                        "warmup_s": t_warm,
                        "recall_at_10": D.recall_at_k(got, want, k),
                        "host_api_qps_including_cache_updates": a.calls * a.batch / t_meas,
                        "admitted_during_measured_calls": adm,
                        # where a call's time goes: the searches' GPU span (events around every slot's pass chain, the
                        # slowest slot) against the host call's wall time (staging, cache updates between calls)
                        "kernel_ms_per_call": kms / a.calls, "wall_ms_per_call": t_meas * 1e3 / a.calls,
                        "config": {"n": a.n, "dim": dim, "metric": "IP", "elem": "f16", "M": M, "efc": efc,
                                   "ef": a.ef, "k": k, "batch": a.batch, "warmup_calls": a.warm,
                                   "measured_calls": a.calls, "pool": pool_n},
                        "note": "one physical GPU unless physical_gpus > 1: read classes exact, xGMI rate not measured"}
                log(json.dumps(line))
                with open(a.out, "a") as f:
                    f.write(json.dumps(line) + "\n")
    for h in opened.values():
        h.close()
    gb.close()


if __name__ == "__main__":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # batches in flight on distinct hardware queues (the box exports 4)
    main()
