#!/usr/bin/env python3
"""BASELINE.json configs at full size on one MI355X, with indexes built by the GPU batch builder (shine_gpu_build).

  cmp    SIFT-shaped 1M x 128, M=16, efC=200: the CPU builder (16 threads) and the GPU builder on the same rows;
           recall@10 at ef=128 of both (fast mode, 10K queries), build times, and the oracle's knn on the GPU-built
           dump against exact mode on a sample (bitwise)
  cfg3     DEEP-shaped 10M x 96, inner product, ef=256, batch 4096 (configs[2])
  cfg4     DEEP-shaped 100M x 96, L2, ef=128, batch 1024 (configs[3]), one replica: 51 GB of rows + lists
  cfg5     TTI-shaped 50M x 200, inner product, fp16 rows, ef=250, batch 1024, Zipf alpha 1.0 query mix (configs[4])
  cfg5_10m the cfg5 shape at 10M records, one replica (the fp16 / d=200 kernel on its own)

Rows are generated on the GPU (shine_amd.datasets.generate_device), the index is built from them in HBM, ground truth
comes from an f32 scan refined in float64, and the timed search reuses tools/config_lines.py's measure(): four batches
in flight, HIP events, algorithmic bytes over the launches' span.  One JSON line per workload and mode.

Usage: python tools/scale_lines.py --which cfg4 [--n 100000000] [--out gpurun_out/scale_lines.jsonl]
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
sys.path.insert(0, str(ROOT / "oracle"))
from bench import host_threads, log  # noqa: E402
from config_lines import Heartbeat, measure  # noqa: E402

WORKLOADS = {
    # name: kind, n, dim, metric, elem, M, efc, ef, batch, zipf alpha (None: plain queries)
    "cfg3": ("deep_like", 10_000_000, 96, 1, 0, 16, 200, 256, 4096, None),
    "cfg4": ("deep_like", 100_000_000, 96, 0, 0, 16, 200, 128, 1024, None),
    "cfg5": ("tti_like", 50_000_000, 200, 1, 1, 16, 200, 250, 1024, 1.0),
    "cfg5_10m": ("tti_like", 10_000_000, 200, 1, 1, 16, 200, 250, 1024, 1.0),
}


def build_gpu(torch, shine_amd, base_t, M, efc, metric, a, label):
    n, dim = base_t.shape
    t0 = time.time()
    with Heartbeat(f"{label}: GPU build {n} x {dim}"):
        gb = shine_amd.GpuBuild(base_t.data_ptr(), M, efc, metric, seed=1234, n=n, dim=dim,
                                batch_fraction=a.batch_fraction, max_batch=a.max_batch)
    wall = time.time() - t0
    st = gb.stats()
    st["wall_s"] = wall
    st["inserts_per_s"] = n / wall
    log(f"{label}: built {n} x {dim} in {wall:.1f}s ({st['batches']} batches, {n / wall / 1e6:.2f} M inserts/s)")
    return gb, st


def queries(torch, D, kind, dim, nq, alpha):
    if alpha is None:
        return D.generate_device(kind, nq, seed=2, d=dim)
    pool = D.generate_device(kind, 500_000, seed=2, d=dim).cpu().numpy()  # skew.py's query pool (500k)
    q, _, _ = D.zipf_query_mix(pool, nq, alpha, seed=3)
    return torch.from_numpy(np.ascontiguousarray(q)).cuda()


def run(name, a):
    import torch
    import shine_amd
    from shine_amd import datasets as D
    kind, n, dim, metric, elem, M, efc, ef, batch, alpha = WORKLOADS[name]
    n = a.n or n
    base_t = D.generate_device(kind, n, seed=1, d=dim)
    # --per-slot: with slots > 1 every slot answers a whole batch per step (global batch = batch x slots), as bench.py's
    # sharded leg does, instead of 1/slots of one batch (a GPU of a sharded node runs full launches)
    bmul = max(int(x) for x in a.slots.split(",")) if a.per_slot else 1
    nq = batch * bmul * a.nbatches
    q = queries(torch, D, kind, dim, nq, alpha)
    with Heartbeat(f"{name}: ground truth"):
        gt = D.ground_truth_device(base_t, q, a.k, metric)
    gb, st = build_gpu(torch, shine_amd, base_t, M, efc, metric, a, name)
    del base_t
    torch.cuda.empty_cache()
    L = shine_amd._lib
    ef0 = int((a.ef or str(ef)).split(",")[0])
    # the oracle's knn on the GPU-built dump (a checker sample, before the replica takes the build's arrays)
    orc = oracle_ref(shine_amd, gb, q, a.k, ef0, dim, M, metric, 8 if name in ("cfg4", "cfg5") else 1,
                     a.cmp_oracle_n) if a.cmp_oracle else None
    if orc is not None and elem != L.ELEM_F32:  # exact mode on f32 rows of the same graph (the oracle's element type)
        with gb.open_ex(1, elem=L.ELEM_F32, gpus=[0]) as ix:
            ix.set_search_mode(L.MODE_EXACT)
            orc["exact"] = ix.knn(orc["q"], a.k, ef0)
    lines = []
    # slots > 1: the same graph as `slots` memory-node dumps under SHINE_PLACE_SHARDED over GPU slots that repeat this
    # box's device (the 8-slot emulation of configs[3]/[4]); every slot answers 1/slots of each batch.  The replica
    # goes last: open() moves the build's arrays into it.
    for slots in sorted({int(s) for s in a.slots.split(",")}, reverse=True):
        if slots == 1:
            idx, placement = gb.open(elem), "replica"
        else:
            idx, placement = gb.open_ex(slots, elem=elem, gpus=[0] * slots, placement="sharded"), "sharded"
        for env in a.envs.split(";"):  # --envs: the same measurement under library tuning hooks (A/B on one build)
            kv = [x.partition("=") for x in env.split(",") if x]
            for k_, _, v_ in kv:
                os.environ[k_] = v_
            for rep in range(a.repeat):  # --repeat: the same measurement again on the same handle (warm-state check)
                gbatch = batch * slots if a.per_slot else batch
                for line in run_measure(torch, idx, name, a, q, gt, gbatch, slots, ef, kind, n, dim, metric, M, efc,
                                        placement, alpha, nq, elem, st):
                    line["repeat"] = rep
                    line["env"] = env
                    lines.append(line)
            for k_, _, _ in kv:
                del os.environ[k_]
        if orc is not None and slots == 1 and "exact" not in orc:  # f32 rows: the measured replica itself
            idx.set_search_mode(L.MODE_EXACT)
            orc["exact"] = idx.knn(orc["q"], a.k, ef0)
        idx.close()
    gb.close()
    if orc is not None:
        res = oracle_compare(orc)
        for line in lines:
            line["oracle"] = res
            line["oracle_equals_exact_on_gpu_dump"] = res["oracle_equals_exact_on_gpu_dump"]
    return lines


def oracle_ref(shine_amd, gb, q, k, ef, dim, M, metric, shards, n_sample):
    """The oracle's knn (the checker; hnsw.hh:253-307) on the GPU-built index's dump images, n_sample queries spread
    over the measured set.  Exact mode on f32 rows of the same graph is compared with it (oracle_compare): ids in heap
    order, distances bitwise, counters."""
    import oracle as O
    qn = q.cpu().numpy()
    sel = np.linspace(0, qn.shape[0] - 1, n_sample).astype(np.int64)
    qs = np.ascontiguousarray(qn[sel])
    t0 = time.time()
    with Heartbeat(f"oracle sample: dump images of {shards} memory nodes"):
        dumps = gb.dumps(shards, copy=False)
    t1 = time.time()
    with Heartbeat(f"oracle sample: {n_sample} queries"):
        I = O.OracleIndex(dumps, dim, M, metric)
        ref = I.knn(qs, k, ef, threads=host_threads())
        I.close()
    del dumps
    return {"q": qs, "ref": ref, "ef": ef, "memory_nodes": shards, "dumps_s": t1 - t0, "oracle_s": time.time() - t1}


def oracle_compare(orc):
    ex = orc["exact"]
    ref_ids, ref_d, ref_qs = orc["ref"]
    same_ids = np.array_equal(ex.ids, ref_ids)
    same_d = np.array_equal(ex.dists.view(np.uint32), ref_d.view(np.uint32))
    same_qs = np.array_equal(ex.qstats[:, :5], ref_qs[:, :5])
    out = {"oracle_equals_exact_on_gpu_dump": bool(same_ids and same_d and same_qs), "queries": int(orc["q"].shape[0]),
           "same_ids_heap_order": float((ex.ids == ref_ids).all(1).mean()),
           "same_dists_bitwise": float((ex.dists.view(np.uint32) == ref_d.view(np.uint32)).all(1).mean()),
           "same_counters": float((ex.qstats[:, :5] == ref_qs[:, :5]).all(1).mean()),
           "exact_rows": "f32", "ef": orc["ef"], "memory_nodes": orc["memory_nodes"], "dumps_s": orc["dumps_s"],
           "oracle_s": orc["oracle_s"]}
    log(f"oracle sample: {json.dumps(out)}")
    return out


def run_measure(torch, idx, name, a, q, gt, batch, slots, ef, kind, n, dim, metric, M, efc, placement, alpha, nq,
                elem, st):
    ns = argparse.Namespace(**{**vars(a), "ef": a.ef or str(ef), "nbatches": a.nbatches})
    lines = []
    for line in measure(torch, idx, name, ns, q, gt, batch, slots, ef):
        line["config"].update({"generator": kind, "n": n, "dim": dim, "metric": "IP" if metric else "L2", "M": M,
                               "efc": efc, "placement": placement, "gpu_slots": [0] * slots,
                               "zipf_alpha": alpha, "queries": nq})
        line["dtype"] = "f16 records, f32 accumulate" if elem == 1 else "f32"
        line["build"] = st
        line["data"] = "synthetic (GPU-generated, seeded); index built in-run on the GPU (shine_gpu_build)"
        log(json.dumps(line))
        lines.append(line)
    return lines


def run_cmp(a):
    """CPU builder vs GPU builder on the same 1M SIFT-shaped rows (VERDICT r3 item 1's acceptance)."""
    import torch
    import shine_amd
    from shine_amd import datasets as D
    import oracle as O
    L = shine_amd._lib
    n, dim, M, efc, ef, k = a.n or 1_000_000, a.cmp_dim, 16, 200, 128, a.k
    metric = a.cmp_metric
    base = getattr(D, a.cmp_kind)(n, seed=1, d=dim)
    q = getattr(D, a.cmp_kind)(10_240, seed=2, d=dim)
    base_t = torch.from_numpy(base).cuda()
    qd = torch.from_numpy(q).cuda()
    gt = D.ground_truth_device(base_t, qd, k, metric)
    t0 = time.time()
    with Heartbeat("cmp: CPU build"):
        cpu_dumps, _ = shine_amd.build(base, M, efc, metric, 1, seed=1234, threads=host_threads())
    cpu_s = time.time() - t0
    line = {"workload": "cmp", "kind": a.cmp_kind, "metric": metric, "n": n, "dim": dim, "M": M, "efc": efc,
            "ef": ef, "queries": int(q.shape[0]), "cpu_build_s": cpu_s, "cpu_build_threads": host_threads()}
    builds = [("cpu", cpu_dumps)]
    for fr in [float(x) for x in a.cmp_fracs.split(",")]:
        a.batch_fraction = fr
        gb, st = build_gpu(torch, shine_amd, base_t, M, efc, metric, a, "cmp")
        label = "gpu" if len(builds) == 1 else f"gpu_frac{fr}"
        line[f"{label}_build"] = st
        builds.append((label, gb.dumps(1)))
        gb.close()
    gpu_dumps = builds[1][1]
    res = {}
    for label, dumps in builds:
        with shine_amd.Index.from_buffers(dumps, dim, M, metric, gpus=[0]) as idx:
            idx.set_search_mode(L.MODE_FAST)
            r = idx.knn(q, k, ef)
            res[label] = r
            line[f"recall_{label}"] = D.recall_at_k(r.ids, gt, k)
            line[f"mean_distcomps_{label}"] = float(r.qstats[:, 0].mean())
            for e2 in (32, 48, 64, 256):
                line[f"recall_{label}_ef{e2}"] = D.recall_at_k(idx.knn(q, k, e2).ids, gt, k)
            if label == "gpu" and a.cmp_oracle:
                idx.set_search_mode(L.MODE_EXACT)
                ex = idx.knn(q[:512], k, ef)
                ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, dim, M, metric).knn(q[:512], k, ef, threads=host_threads())
                line["oracle_equals_exact_on_gpu_dump"] = bool(
                    np.array_equal(ex.ids, ref_ids) and np.array_equal(ex.dists.view(np.uint32), ref_d.view(np.uint32))
                    and np.array_equal(ex.qstats[:, :5], ref_qs[:, :5]))
                line["oracle_sample"] = 512
    line["recall_gap"] = line["recall_cpu"] - line["recall_gpu"]
    gs = shine_amd.graph_stats(gpu_dumps, dim, M)
    line["gpu_graph"] = gs
    line["cpu_graph"] = shine_amd.graph_stats(cpu_dumps, dim, M)
    log(json.dumps(line))
    return [line]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--which", default="cmp")
    p.add_argument("--n", type=int, default=0, help="override the workload's record count")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--nbatches", type=int, default=10)
    p.add_argument("--ef", default="")
    p.add_argument("--modes", default="fast,exact")
    p.add_argument("--inflight", type=int, default=4)
    p.add_argument("--repeat", type=int, default=1)
    p.add_argument("--envs", default="", help="';'-separated variants of comma-separated KEY=VALUE library hooks, "
                                              "measured one after the other on the same handle ('' = defaults)")
    p.add_argument("--per-slot", action="store_true", help="slots > 1: a whole batch per slot per step")
    p.add_argument("--slots", default="1", help="GPU slots per layout, e.g. 1,8: the same graph as a replica and "
                                                "as 8 sharded memory-node dumps on this device")
    p.add_argument("--batch-fraction", type=float, default=0.0)
    p.add_argument("--max-batch", type=int, default=0)
    p.add_argument("--cmp-kind", default="sift_like")
    p.add_argument("--cmp-dim", type=int, default=128)
    p.add_argument("--cmp-metric", type=int, default=0)
    p.add_argument("--cmp-oracle", type=int, default=1,
                   help="cmp: the oracle on 512 queries of the GPU-built dump; cfg*: on --cmp-oracle-n queries")
    p.add_argument("--cmp-oracle-n", type=int, default=64)
    p.add_argument("--cmp-fracs", default="0.02", help="cmp: GPU builds at these batch fractions")
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "scale_lines.jsonl"))
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from config_lines import reserve_streams
    reserve_streams(torch, a.inflight * max(int(s) for s in a.slots.split(",")))  # first streams of the process
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    for name in a.which.split(","):
        for line in (run_cmp(a) if name == "cmp" else run(name, a)):
            print(json.dumps(line), flush=True)
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # batches in flight on distinct hardware queues (the box exports 4)
    main()
