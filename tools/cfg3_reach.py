#!/usr/bin/env python3
"""cfg 3 investigation (VERDICT r01 "What's weak" 4): does recall@10 plateau because of the index or the search?

Builds the cfg-3-shaped index (DEEP-like 96-d inner product, M=16, efC=200) with the parallel builder, then on the
CPU only:
  * graph reachability from the entry point (shine_graph_stats_buffers): records a level-0 search can never reach;
  * the oracle (C++ restatement of HNSW::knn, hnsw.hh:253-307) on a query sample at several ef, recall@10 against
    exact ground truth (f32 scan, top candidates re-ranked in f64).
The oracle is the checker here: this is a diagnostic tool, nothing in the product calls it.

With --gpu it also answers the same queries on the GPU (both search modes, the batch padded to --batch queries
so the launch shape is the config's) and computes the torch ground truth the round-1 config lines used, to tell
which of index, search or ground truth moved the recall.

Usage: python tools/cfg3_reach.py --n 10000000 --threads 8 [--nq 512] [--ef 256,512] [--cache /tmp/cfg3] [--gpu]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT / "oracle"))


def log(msg):
    print(f"[cfg3 {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def exact_gt(base, q, k, metric, chunk=1 << 18, cand=64):
    """Top-k by exact distance: f32 scan keeps `cand` candidates per query, re-ranked in f64 (ties by id)."""
    best_d = np.full((q.shape[0], 0), np.inf, np.float32)
    best_i = np.zeros((q.shape[0], 0), np.int64)
    qn = (q * q).sum(1)
    for s in range(0, base.shape[0], chunk):
        b = base[s:s + chunk]
        ip = q @ b.T
        d = 1.0 - ip if metric == 1 else qn[:, None] + (b * b).sum(1)[None, :] - 2.0 * ip
        c = min(cand, d.shape[1])
        part = np.argpartition(d, c - 1, axis=1)[:, :c]
        best_d = np.concatenate([best_d, np.take_along_axis(d, part, 1)], 1)
        best_i = np.concatenate([best_i, part + s], 1)
        keep = np.argpartition(best_d, min(cand, best_d.shape[1]) - 1, axis=1)[:, :cand]
        best_d = np.take_along_axis(best_d, keep, 1)
        best_i = np.take_along_axis(best_i, keep, 1)
    out = np.empty((q.shape[0], k), np.int64)
    for r in range(q.shape[0]):
        ids = best_i[r]
        x = base[ids].astype(np.float64)
        qq = q[r].astype(np.float64)
        d = 1.0 - x @ qq if metric == 1 else ((x - qq) ** 2).sum(1)
        order = np.lexsort((ids, d))[:k]
        out[r] = ids[order]
    return out


def gpu_check(a, base, dump, q, gt):
    """GPU answers for the same queries (padded to one batch of a.batch) and the torch ground truth."""
    import torch
    import shine_amd
    from shine_amd import datasets as D
    from config_lines import ground_truth
    out = {}
    bt = torch.from_numpy(base).cuda()
    qt0 = torch.from_numpy(q).cuda()
    # the round-1 ground truth: float32 GEMM + topk (what the config lines used then)
    g32 = np.concatenate([torch.topk(qt0[s:s + 256] @ bt.T if a.metric == 1 else
                                     -((qt0[s:s + 256] ** 2).sum(1)[:, None] + (bt * bt).sum(1)[None, :] -
                                       2.0 * (qt0[s:s + 256] @ bt.T)), 10).indices.cpu().numpy()
                          for s in range(0, q.shape[0], 256)])
    out["torch_f32_gt_recall_vs_exact"] = D.recall_at_k(g32, gt, 10)
    g_t = ground_truth(torch, bt, qt0, 10, a.metric)
    out["torch_f64_gt_recall_vs_exact"] = D.recall_at_k(g_t, gt, 10)
    log(f"torch ground truth vs exact: f32 GEMM {out['torch_f32_gt_recall_vs_exact']:.4f}, "
        f"f64 {out['torch_f64_gt_recall_vs_exact']:.4f}")
    del bt
    torch.cuda.empty_cache()
    reps = (a.batch + q.shape[0] - 1) // q.shape[0]
    qb = np.ascontiguousarray(np.tile(q, (reps, 1))[:a.batch])
    qt = torch.from_numpy(qb).cuda()
    with shine_amd.Index.from_buffers([dump], a.dim, a.M, a.metric, gpus=[0]) as idx:
        for mode, name in ((shine_amd.MODE_FAST, "fast"), (shine_amd.MODE_EXACT, "exact")):
            idx.set_search_mode(mode)
            for ef in [int(x) for x in a.ef.split(",")]:
                ids = torch.empty((a.batch, 10), dtype=torch.int32, device="cuda")
                qs = torch.zeros((a.batch, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
                idx.knn_device(qt.data_ptr(), a.batch, 10, ef, ids.data_ptr(), None, qs.data_ptr(),
                               stream=torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                r = ids.cpu().numpy().view(np.uint32)[:q.shape[0]]
                st = qs.cpu().numpy().view(np.uint32)
                rec = D.recall_at_k(r, gt, 10)
                out[f"{name}_ef{ef}"] = {"recall_at_10": rec, "failed": int((st[:, 6] != 0).sum()),
                                         "mean_distcomps": float(st[:q.shape[0], 0].mean())}
                log(f"gpu {name} ef={ef}: recall@10 {rec:.4f} (vs torch gt {D.recall_at_k(r, g_t, 10):.4f}), "
                    f"distcomps {st[:q.shape[0], 0].mean():.0f}")
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--dim", type=int, default=96)
    p.add_argument("--M", type=int, default=16)
    p.add_argument("--efc", type=int, default=200)
    p.add_argument("--metric", type=int, default=1)
    p.add_argument("--gen", default="deep_like")
    p.add_argument("--threads", type=int, default=8)
    p.add_argument("--nq", type=int, default=512)
    p.add_argument("--ef", default="256,512")
    p.add_argument("--cache", default="/tmp/cfg3")
    p.add_argument("--out", default="")
    p.add_argument("--gpu", action="store_true")
    p.add_argument("--batch", type=int, default=4096)
    a = p.parse_args()
    import oracle as O
    import shine_amd
    from shine_amd import datasets as D

    base = getattr(D, a.gen)(a.n, seed=1, d=a.dim)
    cache = Path(a.cache) / f"{a.gen}-{a.n}-{a.dim}-{a.M}-{a.efc}-{a.metric}-t{a.threads}"
    path = cache / shine_amd.dump_name(a.M, a.efc, 0, 1)
    sys.path.insert(0, str(ROOT / "tools"))
    from config_lines import Heartbeat
    if not path.exists():
        t0 = time.time()
        with Heartbeat(f"building {a.n} x {a.dim}"):
            dumps, _ = shine_amd.build(base, a.M, a.efc, a.metric, 1, seed=1234, threads=a.threads)
        log(f"built {a.n} x {a.dim} in {time.time() - t0:.0f}s on {a.threads} threads")
        cache.mkdir(parents=True, exist_ok=True)
        dumps[0].tofile(path)
        del dumps
    dump = np.fromfile(path, dtype=np.uint8)
    t0 = time.time()
    gs = shine_amd.graph_stats([dump], a.dim, a.M)
    log(f"graph stats in {time.time() - t0:.0f}s: {gs}")
    q = getattr(D, a.gen)(a.nq, seed=2, d=a.dim)
    t0 = time.time()
    gt = exact_gt(base, q, 10, a.metric)
    log(f"ground truth in {time.time() - t0:.0f}s")
    I = O.OracleIndex([dump], a.dim, a.M, a.metric)
    res = {"n": a.n, "gen": a.gen, "dim": a.dim, "M": a.M, "efc": a.efc, "metric": a.metric,
           "build_threads": a.threads, "nq": a.nq, "graph": gs, "oracle": []}
    for ef in [int(x) for x in a.ef.split(",")]:
        t0 = time.time()
        ids, dd, qs = I.knn(q, 10, ef, threads=a.threads)
        rec = D.recall_at_k(ids, gt, 10)
        res["oracle"].append({"ef": ef, "recall_at_10": rec, "mean_distcomps": float(qs[:, 0].mean()),
                              "seconds": time.time() - t0})
        log(f"oracle ef={ef}: recall@10 {rec:.4f}, distcomps {qs[:, 0].mean():.0f} ({time.time() - t0:.0f}s)")
    I.close()
    if a.gpu:
        res["gpu"] = gpu_check(a, base, dump, q, gt)
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
