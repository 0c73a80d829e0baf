#!/usr/bin/env python3
"""Measurement lines for the BASELINE.json configs other than the headline one (bench.py measures configs[1]).

Each workload builds its index in-run (parallel HNSW::insert restatement), keeps queries and outputs in HBM, runs a
validation pass (status, recall@10 against exact ground truth computed on the GPU), then times K batches with HIP
events.  One JSON line per workload and search mode is printed and appended to --out.

  cfg3     DEEP-shaped 96-d inner product, ef=256, batch 4096 (configs[2]; N reduced from 10M, see `n`)
  cfg5     TTI-shaped 200-d inner product, records in fp16, Zipf-skewed query mix (alpha 1.0, skew.py:114-164),
           ef=250 (scripts/datasets.py: TTI reaches ~95 % at 250) (configs[4]; N reduced from 50M, one GPU)
  sharded  the bench's SIFT-shaped L2 index as 4 memory-node dumps under SHINE_PLACE_SHARDED over GPU slots [0, 0]
           (one physical GPU: both stripes are local, so this checks the layout's cost, not xGMI)
  cfg5skew cfg5's cache-size-and-skew grid on the sharded layout: hit rate before / after a cache warmup per alpha

Usage: python tools/config_lines.py [--which cfg3,cfg5,sharded] [--n 1000000] [--steps 10]
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
from bench import HBM_PEAK_GBPS, host_threads, log  # noqa: E402

WORKLOADS = {
    # name: generator, dim, metric, elem, M, efc, ef, batch, shards, placement, gpus
    "cfg3": ("deep_like", 96, 1, 0, 16, 200, 256, 4096, 1, "replica", [0]),
    "cfg5": ("tti_like", 200, 1, 1, 16, 200, 250, 1024, 1, "replica", [0]),
    # cfg4-shaped (configs[3]: DEEP L2 sharded over 8 GPUs, ef=128): 8 memory-node dumps over 8 GPU slots; on a
    # one-GPU box the slots repeat device 0 (every stripe its own allocation: the read classes are exact, all local)
    "cfg4": ("deep_like", 96, 0, 0, 16, 200, 128, 1024, 8, "sharded", [0] * 8),
    "sharded": ("sift_like", 128, 0, 0, 16, 200, 128, 1024, 4, "sharded", [0, 0]),
    "sharded1": ("sift_like", 128, 0, 0, 16, 200, 128, 1024, 4, "sharded", [0]),   # one slot: the VM layout alone
    "replica4": ("sift_like", 128, 0, 0, 16, 200, 128, 1024, 4, "replica", [0]),   # same 4 dumps, plain HBM
}


class Heartbeat:
    """Prints a line every 30 s while a long native call (index build, ground truth) runs, so that the GPU box's
    watchdog, which kills a command silent for 3 minutes, sees progress."""

    def __init__(self, what):
        import threading
        self.what, self.stop = what, threading.Event()
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        t0 = time.time()
        while not self.stop.wait(30):
            log(f"{self.what}: {time.time() - t0:.0f}s")

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join()


def ground_truth(torch, base_t, q_t, k, metric):
    """Exact top-k on the GPU in float64.  The round-1 version multiplied in float32, and torch's f32 GEMM on this
    stack does not give exact f32 products: on the 10M DEEP-like index its "ground truth" agreed with the exact one
    at recall 0.875 only (tools/cfg3_reach.py, profiles/r02/cfg3_10m.jsonl), which was the cfg-3 plateau."""
    out = []
    b64 = base_t.double()
    bn = (b64 * b64).sum(1) if metric == 0 else None
    for s in range(0, q_t.shape[0], 256):
        qq = q_t[s:s + 256].double()
        dot = qq @ b64.T
        if metric == 0:
            d = (qq * qq).sum(1)[:, None] + bn[None, :] - 2.0 * dot
            out.append(torch.topk(d, k, largest=False).indices.cpu().numpy())
        else:
            out.append(torch.topk(dot, k, largest=True).indices.cpu().numpy())
    del b64
    return np.concatenate(out)


def build_dumps(name, gen, n, dim, M, efc, metric, shards, a):
    """The workload's memory-node dumps under --cache (built once per box, shared by layouts and cache variants)."""
    import shine_amd
    from shine_amd import datasets as D
    key = hashlib.sha1(f"{n}-{dim}-{M}-{efc}-{shards}-{gen}-v1".encode()).hexdigest()[:12]
    cache = Path(a.cache) / key
    base = getattr(D, gen)(n, seed=1, d=dim)
    paths = [cache / shine_amd.dump_name(M, efc, i, shards) for i in range(shards)]
    if not all(p.exists() for p in paths):
        t0 = time.time()
        with Heartbeat(f"{name}: building {n} x {dim}"):
            dumps, _ = shine_amd.build(base, M, efc, metric, shards, seed=1234, threads=host_threads())
        log(f"{name}: built {n} x {dim} in {time.time() - t0:.1f}s")
        cache.mkdir(parents=True, exist_ok=True)
        for p, d in zip(paths, dumps):
            d.tofile(p)
        del dumps
    return base, paths


def read_classes(qs_h):
    """Record reads of a set of queries by class (qstats words, include/shine_gpu.h).  cache_hit_rate has the
    reference's denominator, every node read (statistics.hh:171-173: on a compute node every read is remote);
    off_stripe_hit_rate counts only the reads of records another GPU holds."""
    import shine_amd
    L = shine_amd._lib
    reads = np.maximum(qs_h[:, L.QS_DISTCOMPS].astype(np.int64) - 1, 0).sum()
    hits = qs_h[:, L.QS_CACHED_VEC].astype(np.int64).sum()
    remote = qs_h[:, L.QS_REMOTE_VEC].astype(np.int64).sum()
    return {"node_reads": int(reads), "cache_hit_rate": float(hits / max(1, reads)),
            "off_stripe_share": float((hits + remote) / max(1, reads)),
            "off_stripe_hit_rate": float(hits / max(1, hits + remote))}


def run(name, a):
    import torch
    import shine_amd
    from shine_amd import datasets as D
    gen, dim, metric, elem, M, efc, ef, batch, shards, placement, gpus = WORKLOADS[name]
    n = a.n
    base, paths = build_dumps(name, gen, n, dim, M, efc, metric, shards, a)
    slots = len(gpus)
    nb = a.nbatches
    if name == "cfg5":  # Zipf-skewed replay of a query pool (skew.py), alpha 1.0
        pool = getattr(D, gen)(50_000, seed=2, d=dim)
        q, _, _ = D.zipf_query_mix(pool, batch * nb, 1.0, seed=3)
        q = np.ascontiguousarray(q)
    else:
        q = getattr(D, gen)(batch * nb, seed=2, d=dim)
    qd = torch.from_numpy(q).cuda()
    dyn = None
    with Heartbeat(f"{name}: ground truth"):
        base_t = torch.from_numpy(base).cuda()
        gt = ground_truth(torch, base_t, qd, a.k, metric)
        if placement == "sharded" and a.dynamic:  # the dynamic-cache stream: a fresh batch every call
            dq = np.ascontiguousarray(getattr(D, gen)(a.dynamic_calls * batch, seed=11, d=dim))
            dyn = (dq, ground_truth(torch, base_t, torch.from_numpy(dq).cuda(), a.k, metric))
        del base_t
    del base
    torch.cuda.empty_cache()
    fracs = [float(x) for x in a.cache_fracs.split(",")] if placement == "sharded" else [0.0]
    lines = []
    for frac in fracs:
        with Heartbeat(f"{name}: opening (cache {frac})"):
            idx = shine_amd.Index.open(paths, dim, M, metric, elem=elem, gpus=gpus, placement=placement, cache=frac)
        if frac > 0 and a.cache_warmup:  # compute_node.cc:116-131: a warmup run fills the cache before measuring
            warm = getattr(D, gen)(a.cache_warmup, seed=5, d=dim)
            with Heartbeat(f"{name}: cache warmup"):
                idx.cache_warmup(warm, a.k, ef, query_ids=np.arange(warm.shape[0], dtype=np.uint32))
        for line in measure(torch, idx, name, a, qd, gt, batch, slots, ef):
            line["config"].update({"generator": gen, "n": n, "dim": dim, "metric": "IP" if metric else "L2", "M": M,
                                   "efc": efc, "shards": shards, "placement": placement, "gpu_slots": gpus,
                                   "cache_fraction": frac, "cache_warmup_queries": a.cache_warmup if frac else 0})
            line["dtype"] = "f16 records, f32 accumulate" if elem else "f32"
            log(json.dumps(line))
            lines.append(line)
        idx.close()
    if dyn is not None:
        lines.append(run_dynamic(name, a, paths, dim, M, metric, elem, gpus, dyn[0], dyn[1], batch, ef))
    return lines


def run_dynamic(name, a, paths, dim, M, metric, elem, gpus, q, gt, batch, ef):
    """The reference's runtime cache (SHINE_CACHE_DYNAMIC: admission, cooling eviction, second chance, applied
    between calls) over a stream of distinct batches through the host API: hit rate per call from an empty cache,
    recall over the whole stream, and the host call rate including the cache updates."""
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    idx = shine_amd.Index.open(paths, dim, M, metric, elem=elem, gpus=gpus, placement="sharded")
    idx.set_search_mode(L.MODE_FAST)
    idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=a.dynamic, seed=1)
    rates, res, t_total = [], [], 0.0
    calls = a.dynamic_calls
    nb = q.shape[0] // batch
    for c in range(calls):
        b = c % nb
        t0 = time.perf_counter()
        r = idx.knn(q[b * batch:(b + 1) * batch], a.k, ef,
                    query_ids=np.arange(c * batch, (c + 1) * batch, dtype=np.uint32))
        t_total += time.perf_counter() - t0
        rates.append(r.stats["node_cache_hits"] / max(1, r.stats["node_reads"]))
        res.append(r.ids)
    idx.close()
    line = {"workload": name, "search_mode": "fast", "cache_policy": "dynamic", "cache_ratio_percent": a.dynamic,
            "calls": calls, "batch": batch, "distinct_batches": nb, "hit_rate_per_call": rates,
            "cache_hit_rate_last": rates[-1],
            "recall_at_10": D.recall_at_k(np.concatenate(res), np.concatenate([gt[(c % nb) * batch:(c % nb + 1) * batch]
                                                                                for c in range(calls)]), a.k),
            "host_api_qps_including_cache_updates": calls * batch / t_total,
            "note": "hit rate = cached record reads / all record reads (statistics.hh:171-173); the cache is updated "
                    "between calls on the host (cache.h RecordCache) and the arena on the GPU"}
    log(json.dumps(line))
    return line


_STREAMS: list = []


def reserve_streams(torch, n: int):
    """n HIP streams created directly (bench.hip_streams) on the first call — made before any other stream of the
    process, they take consecutive hardware queues of HIP's round-robin — and the same streams on every later call."""
    if len(_STREAMS) < n:
        from bench import hip_streams
        _STREAMS.extend(hip_streams(torch, n - len(_STREAMS), torch.cuda.current_device()))
    return _STREAMS[:n]


def measure(torch, idx, name, a, qd, gt, batch, slots, ef, nb=None):
    """Validation pass, then timed batches on the device (slot s answers rows [s*per, (s+1)*per) of each batch)."""
    import shine_amd
    from shine_amd import datasets as D
    info = idx.info()
    nb = nb or a.nbatches
    ids = torch.empty((nb, batch, a.k), dtype=torch.int32, device="cuda")
    dists = torch.empty((nb, batch, a.k), dtype=torch.float32, device="cuda")
    qs = torch.zeros((nb, batch, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    # a.inflight batches in flight per slot (step i on stream set i % inflight), as bench.py does, on the process's
    # reserved streams (reserve_streams): torch's stream pool, or streams created after the index's own, can hand two
    # batches one hardware queue, and then they run back to back (cfg5-shaped 10M: 1.41 M against 2.33 M QPS,
    # profiles/r04/two_choice_ab_warm.jsonl, scale_10m_v8_streams.jsonl)
    flat = reserve_streams(torch, a.inflight * slots)
    streams = [flat[i * slots:(i + 1) * slots] for i in range(a.inflight)]
    per = batch // slots  # slot s answers rows [s*per, (s+1)*per) of each batch (id % G in the host API)

    def step(i, rec=None):
        b = i % nb
        st = streams[i % a.inflight]
        for s in range(slots):
            lo, hi = s * per, (s + 1) * per if s < slots - 1 else batch
            if rec is not None:
                rec[s][0].record(st[s])
            idx.knn_device(qd[b * batch + lo:b * batch + hi].data_ptr(), hi - lo, a.k, ef, ids[b, lo:hi].data_ptr(),
                           dists[b, lo:hi].data_ptr(), qs[b, lo:hi].data_ptr(), stream=st[s].cuda_stream,
                           gpu_slot=s)
            if rec is not None:
                rec[s][1].record(st[s])

    lines = []
    efs = [int(x) for x in a.ef.split(",")] if a.ef else [ef]
    modes = [m for m in (("fast", shine_amd.MODE_FAST), ("exact", shine_amd.MODE_EXACT)) if m[0] in a.modes.split(",")]
    def reset(ef):
        # every run starts from the same learned state (--envs A/B on one handle): one small call per stream at another
        # ef drops each stream's table floor and the slot's recent worst queries (capi.cc enqueue_search), so a variant
        # measured earlier cannot size the next one's tables
        for st in streams:
            for s in range(slots):
                n = min(64, per)
                idx.knn_device(qd[:n].data_ptr(), n, a.k, ef + 1, ids[0, :n].data_ptr(), dists[0, :n].data_ptr(),
                               qs[0, :n].data_ptr(), stream=st[s].cuda_stream, gpu_slot=s)
        torch.cuda.synchronize()

    for ef, (mode_name, mode) in [(e, m) for e in efs for m in modes]:
        idx.set_search_mode(mode)
        reset(ef)
        for i in range(nb):
            step(i)
        torch.cuda.synchronize()
        qs_h = qs.cpu().numpy().view(np.uint32).reshape(-1, shine_amd.QS_WORDS).copy()
        bad = int((qs_h[:, 6] != 0).sum())
        res = ids.cpu().numpy().view(np.uint32).reshape(-1, a.k)
        recall = D.recall_at_k(res, gt, a.k)
        bq = [idx.algorithmic_bytes(qs_h[b * batch:(b + 1) * batch]) for b in range(nb)]
        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(slots)]
               for _ in range(a.steps)]
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i, evs[i])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern = [max(s.elapsed_time(e) for s, e in ev) for ev in evs]  # the slots run concurrently
        span = max(evs[0][0][0].elapsed_time(e) for ev in evs for _, e in ev)  # first start to last end
        byts = [bq[(a.warmup + i) % nb] for i in range(a.steps)]
        achieved = sum(byts) / (span / 1e3) / 1e9  # launches overlap when batches are in flight
        line = {
            "workload": name, "search_mode": mode_name, "value": a.steps * batch / el, "unit": "queries/s",
            "ms_per_batch": el * 1e3 / a.steps, "avg_launch_ms": float(np.mean(kern)),
            "span_ms_per_batch": span / a.steps, "batches_in_flight": a.inflight, "recall_at_10": recall,
            "failed_queries": bad, "mean_distcomps": float(qs_h[:, 0].mean()),
            # nodes a query marks visited (upper levels + level 0): what its LDS visited table must hold
            "visited_p99": float(np.percentile(qs_h[:, 1].astype(np.int64) + qs_h[:, 2], 99)),
            "visited_max": int((qs_h[:, 1].astype(np.int64) + qs_h[:, 2]).max()),
            "queries_with_ties": float((qs_h[:, 5] > 0).mean()) if mode_name == "fast" else None,
            "reads": read_classes(qs_h),
            "config": {"ef": ef, "k": a.k, "batch": batch, "device_bytes_per_gpu": info["device_bytes"],
                       "id_space": info["id_space"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "algorithmic_bytes_per_batch": float(np.mean(byts))},
            "data": "synthetic, random-seeded; index built in-run",
        }
        lines.append(line)
    return lines


def run_skew(a):
    """cfg5's skew experiment (scripts/exp_cache_size_and_skew.py: Zipf alpha 0-1.5, cache 5 % of the index) on the
    sharded layout: the TTI-shaped fp16 index as 8 memory-node dumps over 8 GPU slots (repeated device ids on a
    one-GPU box: every stripe is a separate allocation, so the read classes are exact, but all reads are local HBM).
    Per alpha: a fresh open with a 5 % cache fraction, the static (in-degree) ranking's hit rate, a cache warmup on
    the warmup split (shine_cache_warmup, compute_node.cc:116-131), then the measured split's hit rate, read classes,
    recall, and its device-timed QPS and roofline fraction; then the same stream under the reference's runtime
    policy (SHINE_CACHE_DYNAMIC) from an empty cache.  Results must not change with the cache: same_ids."""
    import torch
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    gen, dim, metric, elem, M, efc, ef, shards = "tti_like", 200, 1, 1, 16, 200, 250, 8
    n = a.n
    base, paths = build_dumps("skew", gen, n, dim, M, efc, metric, shards, a)
    pool = getattr(D, gen)(20_000, seed=2, d=dim)
    base_t = torch.from_numpy(base).cuda()
    del base
    lines = []
    batch = 1024
    for alpha in [float(x) for x in a.alphas.split(",")]:
        q, warm, _ = D.zipf_query_mix(pool, 3 * batch, alpha, split=batch, seed=9)
        q, warm = np.ascontiguousarray(q), np.ascontiguousarray(warm)
        qd = torch.from_numpy(q).cuda()
        with Heartbeat("skew: ground truth"):
            gt = ground_truth(torch, base_t, qd, a.k, metric)
        qid = np.arange(q.shape[0], dtype=np.uint32)
        with Heartbeat("skew: opening"):
            idx = shine_amd.Index.open(paths, dim, M, metric, elem=elem, gpus=[0] * shards, placement="sharded",
                                       cache=0.05)
        idx.set_search_mode(L.MODE_FAST)
        r0 = idx.knn(q, a.k, ef, query_ids=qid)
        with Heartbeat("skew: warmup"):
            idx.cache_warmup(warm, a.k, ef, query_ids=np.arange(warm.shape[0], dtype=np.uint32))
        r1 = idx.knn(q, a.k, ef, query_ids=qid)
        timed = measure(torch, idx, "cfg5", argparse.Namespace(**{**vars(a), "modes": "fast", "ef": ""}), qd, gt,
                        batch, shards, ef, nb=q.shape[0] // batch)[0]
        idx.close()

        def rate(r):  # off-stripe reads only
            h, m = r.stats["cache_hits"], r.stats["cache_misses"]
            return h / max(1, h + m)

        dyn = {}
        if a.dynamic:
            with shine_amd.Index.open(paths, dim, M, metric, elem=elem, gpus=[0] * shards,
                                      placement="sharded") as di:
                di.set_search_mode(L.MODE_FAST)
                di.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=a.dynamic, seed=1)
                rates = []
                # a fresh Zipf-drawn batch every call (repeats come from the skew itself, not from replaying batches)
                sq, _, _ = D.zipf_query_mix(pool, a.dynamic_calls * batch, alpha, seed=13)
                stream = [np.ascontiguousarray(sq[c * batch:(c + 1) * batch]) for c in range(a.dynamic_calls)]
                for c in range(a.dynamic_calls):
                    qq = stream[c]
                    r = di.knn(qq, a.k, ef, query_ids=np.arange(c * batch, c * batch + qq.shape[0], dtype=np.uint32))
                    rates.append(r.stats["node_cache_hits"] / max(1, r.stats["node_reads"]))
            dyn = {"cache_ratio_percent": a.dynamic, "calls": a.dynamic_calls, "hit_rate_per_call": rates}

        line = {"workload": "cfg5-skew", "alpha": alpha, "cache_fraction": 0.05, "gpu_slots": shards,
                "off_stripe_hit_rate_static": rate(r0), "off_stripe_hit_rate_warmed": rate(r1),
                "cache_hit_rate_static": r0.stats["node_cache_hits"] / max(1, r0.stats["node_reads"]),
                "cache_hit_rate_warmed": r1.stats["node_cache_hits"] / max(1, r1.stats["node_reads"]),
                "remote_share_static": r0.stats["remote_reads_in_bytes"] / max(1, r0.stats["algorithmic_bytes"]),
                "remote_share_warmed": r1.stats["remote_reads_in_bytes"] / max(1, r1.stats["algorithmic_bytes"]),
                "recall_at_10": D.recall_at_k(r1.ids, gt, a.k), "same_ids": bool((r0.ids == r1.ids).all()),
                "value": timed["value"], "unit": "queries/s", "ms_per_batch": timed["ms_per_batch"],
                "recall_at_10_device": timed["recall_at_10"], "reads_device": timed["reads"],
                "roofline": timed["roofline"], "dynamic_cache": dyn,
                "config": {"generator": gen, "n": n, "dim": dim, "metric": "IP", "elem": "f16", "M": M, "efc": efc,
                           "ef": ef, "k": a.k, "batch": batch, "queries": int(q.shape[0]),
                           "warmup_queries": int(warm.shape[0]), "batches_in_flight": a.inflight},
                "note": "one physical GPU: the read classes (local / cached / remote) are exact, the xGMI rate is not "
                        "measured"}
        log(json.dumps(line))
        lines.append(line)
    return lines


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--which", default="cfg3,cfg5,sharded")
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--nbatches", type=int, default=4)
    p.add_argument("--ef", default="", help="comma list overriding the workload's ef (recall / QPS trade-off)")
    p.add_argument("--modes", default="fast,exact")
    p.add_argument("--inflight", type=int, default=4, help="batches in flight per GPU slot (HIP streams)")
    p.add_argument("--cache", default=os.environ.get("SHINE_CFG_CACHE", "/tmp/shine_cfg"))
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "config_lines.jsonl"))
    p.add_argument("--alphas", default="0,0.5,1.0,1.5", help="cfg5skew: Zipf exponents")
    p.add_argument("--cache-fracs", default="0,0.05", help="sharded workloads: cache fractions measured")
    p.add_argument("--cache-warmup", type=int, default=1024,
                   help="queries of the warmup run that ranks a non-empty cache (0: static in-degree ranking)")
    p.add_argument("--dynamic", type=float, default=5.0,
                   help="sharded workloads: also stream batches under SHINE_CACHE_DYNAMIC at this ratio % (0: off)")
    p.add_argument("--dynamic-calls", type=int, default=12)
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    for name in a.which.split(","):
        for line in (run_skew(a) if name == "cfg5skew" else run(name, a)):
            print(json.dumps(line), flush=True)
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
