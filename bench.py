#!/usr/bin/env python3
"""bench.py — QPS at recall@10 >= 0.95 on a SIFT1M-shaped index (BASELINE.json configs[1]).

Workload (one "step" = one batch): 1,024 queries through HNSW::knn (k=10, ef=128) against a 1M x 128-d L2 index
built with M=16, efC=200 by the parallel restatement of HNSW::insert, in the reference's dump layout.  Data are
synthetic SIFT-shaped vectors (shine_amd.datasets.sift_like; no datasets can be fetched).  Queries and outputs
are resident in HBM when the timed region starts; value = queries / wall time over exactly K steps.  Two batches
are in flight per GPU (--inflight; step i is enqueued on HIP stream i % 2), as a serving loop keeps them: the
last, longest queries of one batch overlap the first of the next instead of leaving CUs idle.

Multi-GPU (torchrun, one process per GPU): every rank holds a full replica of the 0.75 GiB index and answers its
own batches (queries split id % G, read_data.hh:57-58) — weak scaling, no data-path collective.  Rank 0 builds
the index once and shares the dump files; the max over ranks of the timed wall time gives `value`.

Also reported: `roofline` for the search kernel (algorithmic bytes of the K launches / their GPU span from HIP
events vs 8 TB/s; `avg_launch_ms` is the per-launch event time, which rocprofv3's average duration matches)
and `cpu_baseline` (the CPU oracle — a C++ restatement of the reference's knn — on the host cores, bounded
sample, rank 0 at N=1 only).
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

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_threads():
    """This process's CPU share: OMP_NUM_THREADS when the launcher sets it (the GPU box grants 16 CPUs per GPU
    while sched_getaffinity lists the whole machine), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except Exception:
        return os.cpu_count() or 1


def rank_queries(pool: np.ndarray, rank: int, world: int, n: int) -> np.ndarray:
    """This rank's queries: ids ≡ rank (mod world) of the common pool, as compute nodes split them
    (read_data.hh:57-58: id % num_clients == client_id)."""
    return np.ascontiguousarray(pool[rank::world][:n])


def prepare_dumps(paths, rank: int, dist, build):
    """Rank 0 builds and writes the memory-node dumps (atomically, via rename) unless they exist; every rank waits
    at a barrier before reading them."""
    if rank == 0 and not all(p.exists() for p in paths):
        dumps = build()
        paths[0].parent.mkdir(parents=True, exist_ok=True)
        for p, d in zip(paths, dumps):
            tmp = p.with_suffix(".tmp")
            d.tofile(tmp)
            tmp.rename(p)
        del dumps
    if dist:
        dist.barrier()


def max_over_ranks(x: float, dist, device: str) -> float:
    """The job's wall time is the slowest rank's (compute_node.cc:549-556 takes the max over compute nodes)."""
    if not dist:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--nbatches", type=int, default=10, help="distinct query batches per rank (cycled)")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--ef", type=int, default=128)
    p.add_argument("--M", type=int, default=16)
    p.add_argument("--efc", type=int, default=200)
    p.add_argument("--shards", type=int, default=1, help="memory-node dumps the index is spread over")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of the CPU-baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--inflight", type=int, default=2,
                   help="query batches in flight per GPU, each on its own HIP stream (step i runs on stream i %% S), "
                        "so one batch's last queries overlap the next batch's first")
    p.add_argument("--ef-sweep", default="32,48,64,96",
                   help="extra ef values timed in fast mode at N=1 (recall/QPS trade-off; not the headline value)")
    p.add_argument("--mode", choices=["fast", "exact", "both"], default="both",
                   help="search mode(s); the first one measured gives `value` (fast, then exact with 'both')")
    p.add_argument("--cache", default=os.environ.get("SHINE_BENCH_CACHE", "/tmp/shine_bench"))
    p.add_argument("--pmc-json", default=str(ROOT / "profiles" / "r01" / "bench_fast_v6_pmc.json"),
                   help="per-launch HBM bytes of the search kernel measured by rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                        "passes of this bench (tools/pmc.py; tools/gpu_round.sh)")
    return p.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import shine_amd
    from shine_amd import datasets as D

    key = hashlib.sha1(f"{a.n}-{a.dim}-{a.M}-{a.efc}-{a.shards}-sift_like-v3".encode()).hexdigest()[:12]
    cache = Path(a.cache) / key
    t0 = time.time()
    base = D.sift_like(a.n, seed=1, d=a.dim)
    log(f"rank {rank}: generated base {base.shape} in {time.time() - t0:.1f}s")
    paths = [cache / "dump" / shine_amd.dump_name(a.M, a.efc, i, a.shards) for i in range(a.shards)]

    def build():
        t0 = time.time()
        dumps, bdc = shine_amd.build(base, a.M, a.efc, shine_amd.METRIC_L2, a.shards, seed=1234,
                                     threads=host_threads())
        log(f"built index: {sum(d.size for d in dumps) / 2**20:.0f} MiB in {time.time() - t0:.1f}s "
            f"({host_threads()} threads, {bdc} distcomps)")
        return dumps

    prepare_dumps(paths, rank, dist, build)
    idx = shine_amd.Index.open(paths, a.dim, a.M, shine_amd.METRIC_L2, gpus=[local])
    info = idx.info()
    log(f"rank {rank}: index on GPU {local}: {info['num_nodes']} nodes, max level {info['max_level']}, "
        f"{info['device_bytes'] / 2**20:.0f} MiB")

    # queries: rank r takes ids ≡ r (mod G) of a common pool (read_data.hh:57-58)
    nq_rank = a.batch * a.nbatches
    pool = D.sift_like(nq_rank * world, seed=2, d=a.dim)
    q = rank_queries(pool, rank, world, nq_rank)
    qd = torch.from_numpy(q).cuda()
    ids = torch.empty((a.nbatches, a.batch, a.k), dtype=torch.int32, device="cuda")
    dists = torch.empty((a.nbatches, a.batch, a.k), dtype=torch.float32, device="cuda")
    qs = torch.zeros((a.nbatches, a.batch, 8), dtype=torch.int32, device="cuda")
    # real streams (the C ABI reads a NULL stream as "the handle's own stream"); the index keeps device scratch per
    # stream, so batches on different streams run concurrently
    if a.nbatches < a.inflight:
        raise SystemExit("--nbatches must be >= --inflight (batches in flight write distinct output buffers)")
    streams = [torch.cuda.Stream() for _ in range(max(1, a.inflight))]
    torch.cuda.set_stream(streams[0])

    def step(i, rec=None, ef=None):
        b = i % a.nbatches
        stream = streams[i % len(streams)]
        if rec is not None:
            rec[0].record(stream)
        idx.knn_device(qd[b * a.batch:(b + 1) * a.batch].data_ptr(), a.batch, a.k, ef or a.ef, ids[b].data_ptr(),
                       dists[b].data_ptr(), qs[b].data_ptr(), stream=stream.cuda_stream)
        if rec is not None:
            rec[1].record(stream)

    # ground truth on the GPU (exact: integer-valued data keep every f32 partial sum < 2^24)
    bt = torch.from_numpy(base).cuda()
    bn = (bt * bt).sum(1)
    gt = []
    for s in range(0, nq_rank, 256):
        qq = qd[s:s + 256]
        dd = (qq * qq).sum(1)[:, None] + bn[None, :] - 2.0 * (qq @ bt.T)
        gt.append(torch.topk(dd, a.k, largest=False).indices.cpu().numpy())
    del bt, bn
    gt = np.concatenate(gt)

    def run_mode(mode):
        """Validation pass over every batch (status, recall, algorithmic bytes), warmup, then exactly K timed
        steps between barriers; returns the measurements."""
        idx.set_search_mode(mode)
        for i in range(a.nbatches):
            step(i)
        torch.cuda.synchronize()
        qs_h = qs.cpu().numpy().view(np.uint32).reshape(-1, 8).copy()
        n_bad = int((qs_h[:, 6] != 0).sum())
        if n_bad:
            raise SystemExit(f"{n_bad} queries did not complete (status {np.unique(qs_h[:, 6])})")
        bq_batch = [idx.algorithmic_bytes(qs_h[b * a.batch:(b + 1) * a.batch]) for b in range(a.nbatches)]
        res = ids.cpu().numpy().view(np.uint32).reshape(-1, a.k).copy()
        recall = D.recall_at_k(res, gt, a.k)
        log(f"rank {rank}: mode {mode}: recall@{a.k} = {recall:.4f} over {nq_rank} queries; mean distcomps "
            f"{qs_h[:, 0].mean():.0f}, lists L0 {qs_h[:, 4].mean():.1f}")
        for i in range(a.warmup):
            step(i)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i, evs[i])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        elapsed = max_over_ranks(t1 - t0, dist, "cuda")
        kern_ms = [s.elapsed_time(e) for s, e in evs]
        span_ms = max(evs[0][0].elapsed_time(e) for _, e in evs)  # first launch's start to the last one's end
        bytes_steps = [bq_batch[(a.warmup + i) % a.nbatches] for i in range(a.steps)]
        return dict(elapsed=elapsed, kern_ms=kern_ms, span_ms=span_ms, bytes_steps=bytes_steps, recall=recall,
                    qs=qs_h, ids=res)

    modes = ["fast", "exact"] if a.mode == "both" else [a.mode]
    runs = {m: run_mode(shine_amd.MODE_FAST if m == "fast" else shine_amd.MODE_EXACT) for m in modes}
    head = runs[modes[0]]
    elapsed, kern_ms, bytes_steps, recall, qs_h = (head[x] for x in ("elapsed", "kern_ms", "bytes_steps", "recall", "qs"))
    # launches overlap when batches are in flight on several streams: the rate is the K launches' algorithmic bytes
    # over their GPU span (HIP events); with one stream the span is the sum of the launch times
    span_ms = head["span_ms"]
    achieved = sum(bytes_steps) / (span_ms / 1e3) / 1e9  # GB/s
    avg_launch_ms = float(np.mean(kern_ms))
    mode_report = {}
    for m, r in runs.items():
        mode_report[m] = {"value": a.steps * a.batch * world / r["elapsed"], "ms_per_step": r["elapsed"] * 1e3 / a.steps,
                          "avg_launch_ms": float(np.mean(r["kern_ms"])), "recall_at_10": r["recall"]}
        if m == "fast":
            mode_report[m]["queries_with_ties"] = float((r["qs"][:, 5] > 0).mean())
    if "fast" in runs and "exact" in runs:
        same = (np.sort(runs["fast"]["ids"], 1) == np.sort(runs["exact"]["ids"], 1)).all(1)
        mode_report["fast"]["same_ids_as_exact"] = float(same.mean())
        clean = runs["fast"]["qs"][:, 5] == 0
        mode_report["fast"]["tie_free_same_ids_as_exact"] = float(same[clean].mean()) if clean.any() else None

    # recall / QPS trade-off of the fast kernel at other ef (the metric is "QPS at recall@10 >= 0.95"); the
    # headline value stays at the config's ef
    sweep = []
    if world == 1 and a.ef_sweep:
        idx.set_search_mode(shine_amd.MODE_FAST)
        for ef in sorted({int(x) for x in a.ef_sweep.split(",") if x.strip()}):
            if not (a.k <= ef <= 256) or ef == a.ef:
                continue
            for i in range(a.nbatches):
                step(i, ef=ef)
            torch.cuda.synchronize()
            qs_e = qs.cpu().numpy().view(np.uint32).reshape(-1, 8)
            if (qs_e[:, 6] != 0).any():
                raise SystemExit(f"ef={ef}: queries did not complete")
            rec_e = D.recall_at_k(ids.cpu().numpy().view(np.uint32).reshape(-1, a.k).copy(), gt, a.k)
            for i in range(a.warmup):
                step(i, ef=ef)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                step(a.warmup + i, ef=ef)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            sweep.append({"ef": ef, "value": a.steps * a.batch / el, "ms_per_step": el * 1e3 / a.steps,
                          "recall_at_10": rec_e})
            log(f"ef sweep: ef={ef} recall@{a.k}={rec_e:.4f} {a.steps * a.batch / el / 1e6:.2f}M QPS")
        if "fast" in runs:
            sweep.append({"ef": a.ef, "value": mode_report["fast"]["value"],
                          "ms_per_step": mode_report["fast"]["ms_per_step"], "recall_at_10": runs["fast"]["recall"]})
        sweep.sort(key=lambda x: x["ef"])

    traffic, traffic_src = None, None
    if a.pmc_json and Path(a.pmc_json).exists():
        pmc = json.loads(Path(a.pmc_json).read_text())
        if any(k.startswith("void shine::(anonymous namespace)::search_fast_kernel<128, 0, float, 2,") for k in pmc.get("kernels", [])):
            traffic = pmc.get("hbm_bytes_per_launch")
            traffic_src = str(Path(a.pmc_json).relative_to(ROOT)) if Path(a.pmc_json).is_relative_to(ROOT) else a.pmc_json

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(paths, q, a, recall)

    if rank == 0:
        total_q = a.steps * a.batch * world
        out = {
            "metric": "QPS at recall@10>=0.95, SIFT1M d=128 batch=1024",
            "value": total_q / elapsed,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic SIFT-shaped (integer-valued f32, 1M x 128), random-seeded; index built in-run",
            "recall_at_10": recall,
            "search_mode": modes[0],
            "modes": mode_report,
            "ef_sweep": sweep or None,
            "best_at_recall_0.95": max((x for x in sweep if x["recall_at_10"] >= 0.95), key=lambda x: x["value"],
                                       default=None),
            "config": {"workload": "SIFT1M-shaped L2 knn, M=16 efC=200 ef=128 k=10", "n": a.n, "dim": a.dim,
                       "global_batch": a.batch * world, "batch_per_gpu": a.batch, "M": a.M, "efc": a.efc,
                       "ef": a.ef, "k": a.k, "shards": a.shards, "parallelism": f"replica{world}",
                       "batches_in_flight": len(streams)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": ("search_fast_kernel<128,L2,f32,R=2,P=2>" if modes[0] == "fast"
                                    else "search_kernel<128,L2,f32,0>"), "avg_launch_ms": avg_launch_ms,
                         "span_ms_per_launch": span_ms / a.steps, "batches_in_flight": len(streams),
                         "achieved_basis": "algorithmic bytes of the K timed launches / their GPU span (first "
                                           "launch start to last launch end, HIP events on the launch streams)",
                         "algorithmic_bytes_per_launch": float(np.mean(bytes_steps)),
                         "mean_distcomps_per_query": float(qs_h[:, 0].mean())},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    idx.close()
    if dist:
        dist.destroy_process_group()


def cpu_baseline(paths, q, a, gpu_recall):
    """The oracle (C++ restatement of the reference's knn) on this host's cores, same dump, same queries."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    dumps = [np.fromfile(p, dtype=np.uint8) for p in paths]
    I = O.OracleIndex(dumps, a.dim, a.M, 0)
    th = host_threads()
    n = min(q.shape[0], 512)
    t0 = time.perf_counter()
    I.knn(q[:n], a.k, a.ef, threads=th)
    probe = time.perf_counter() - t0
    reps = max(1, int(a.cpu_seconds / max(probe, 1e-3)))
    t0 = time.perf_counter()
    done = 0
    for r in range(reps):
        s = (r * n) % max(1, q.shape[0] - n + 1)
        I.knn(q[s:s + n], a.k, a.ef, threads=th)
        done += n
    el = time.perf_counter() - t0
    I.close()
    log(f"cpu baseline: {done} queries in {el:.1f}s on {th} threads")
    return {"value": done / el, "unit": "queries/s", "cores": th, "kind": "port",
            "sample": f"{done} queries (batches of {n} from the bench's query set, k={a.k}, ef={a.ef}) on the "
                      f"same dump, {th} threads, ~{a.cpu_seconds:.0f}s"}


if __name__ == "__main__":
    main()
