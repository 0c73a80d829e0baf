#!/usr/bin/env python3
"""bench.py — QPS at recall@10 >= 0.95 on a SIFT1M-shaped index (BASELINE.json configs[1]).

Workload (one "step" = one batch): 1,024 queries through HNSW::knn (k=10, ef=128) against a 1M x 128-d L2 index
built with M=16, efC=200 in-run by the GPU batch builder (--builder cpu: the parallel restatement of HNSW::insert),
in the reference's dump layout.  Data are
synthetic SIFT-shaped vectors (shine_amd.datasets.sift_like; no datasets can be fetched).  Queries and outputs
are resident in HBM when the timed region starts; value = queries / wall time over exactly K steps.  Four batches
are in flight per GPU (--inflight; step i is enqueued on HIP stream i % 4, each on a hardware queue of its own),
as a serving loop keeps them: the last, longest queries of one batch overlap the next batches' first ones
instead of leaving CUs idle (profiles/r02/inflight_scan_*.jsonl: 2 → 4 in flight is +27 % at ef = 128).

Multi-GPU (torchrun, one process per GPU): every rank holds a full replica of the 0.75 GiB index and answers its
own batches (queries split id % G, read_data.hh:57-58) — weak scaling, no data-path collective.  Rank 0 builds
the index once and shares the dump files; the max over ranks of the timed wall time gives `value`.

Also reported: `roofline` for the search kernel (algorithmic bytes of the K launches / their GPU span from HIP
events vs 8 TB/s; `avg_launch_ms` is the per-launch event time, which rocprofv3's average duration matches),
`value_host_to_host` (SURVEY §8d's query phase: queries and results in pinned host memory that the kernels read and
write over PCIe, K steps, batches in flight as above; `value_host_to_host_copies` the same with copy-engine H2D / D2H;
`value_host_api` is the drop-in C-ABI host call over the rank's whole query set per call, which the library runs as
chunks in flight, two calls kept in flight through shine_knn_batch_async / shine_wait; `value_host_api_sync` the
synchronous shine_knn_batch the same way, one call at a time; `value_host_api_per_batch` that call one batch at a time)
and `cpu_baseline` (the CPU oracle — a C++ restatement of the reference's knn — built with the reference's flags on
the host that runs it, on the host cores, bounded sample, rank 0 at N=1 only).

Row storage: `value` is measured on f32 rows (the reference's records).  `other_rows` times the same fast-mode
search on the narrowest lossless rows (u8: SIFT-shaped components are byte values, as in the reference's .u8bin
inputs) and checks that ids, distances and counters are bitwise the same; it is 4x fewer bytes per distance.

--placement sharded (one process, not torchrun) runs the cfg-4-shaped sharded leg instead: a DEEP-shaped 96-d L2
index as 8 memory-node dumps over --slots GPU slots (slot s on GPU s % device_count; memory node m on slot m % S),
every batch split id % S over the slots, and reports the share of reads that left a slot's stripe (xGMI) and the
bandwidth bound that share implies.
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

# Batches in flight only overlap on distinct hardware queues.  HIP maps streams to its GPU_MAX_HW_QUEUES queues (4 by
# default, and the GPU boxes export 4) round-robin in creation order, and torch's stream pool handed this bench's
# four streams two queues (rocprofv3 kernel trace: queue ids 3 and 4 only), so pairs of batches ran back to back:
# 4.88 M QPS at ef = 128 against 6.23 M with 8 queues (profiles/r02/hwq_streams.txt).  The bench therefore creates its
# in-flight streams itself, directly through HIP and before any other stream of the process (`hip_streams`), so the
# round-robin hands them distinct queues under the box's own setting; the JSON line records that setting.
HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ROW_NAMES = {0: "f32", 1: "f16", 2: "u8", 3: "i8"}  # shine_index_info.elem
KERNEL_TYPE = {"f32": "float", "f16": "__half", "u8": "unsigned char", "i8": "signed char"}  # rocprof kernel names


def hip_streams(torch, n: int, device: int):
    """n non-blocking HIP streams created directly (hipStreamCreateWithFlags), wrapped as torch ExternalStreams.
    Created first in the process, they take n distinct hardware queues of the round-robin (n <= GPU_MAX_HW_QUEUES)."""
    import ctypes
    torch.cuda.set_device(device)
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    out = []
    for _ in range(n):
        s = ctypes.c_void_p()
        rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1))  # hipStreamNonBlocking
        if rc != 0:
            raise SystemExit(f"hipStreamCreateWithFlags failed: {rc}")
        out.append(torch.cuda.ExternalStream(s.value, device=torch.device("cuda", device)))
    return out


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_threads():
    """This process's CPU share: OMP_NUM_THREADS when the launcher sets it (the GPU box grants 16 CPUs per GPU
    while sched_getaffinity lists the whole machine), else the affinity mask."""
    try:
        aff = max(1, len(os.sched_getaffinity(0)))
    except Exception:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = int(env)
        # torchrun sets OMP_NUM_THREADS=1 for every rank unless the caller set it: rank 0's one-off index build (the
        # others wait at a barrier) would then run on one thread; it builds for the whole node, so it takes the
        # node's share (16 CPUs per GPU on this pool) instead
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        if n == 1 and local_world > 1 and os.environ.get("TORCHELASTIC_RUN_ID"):
            return max(1, min(aff, 16 * local_world))
        return n
    return aff


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


def check_same_index(dist, torch, info, world: int, rank: int, device: str):
    """The entry-point all-gather (RCCL on GPUs, gloo in the CPU test; once, outside the timed region): every compute
    node reads the entry point from memory node 1 (rdma_reads.hh:74-99) — here every rank gathers every other's
    (entry uid, level, records) and checks that all serve the same index before any query runs."""
    mine = torch.tensor([info["entry_uid"], info["max_level"], info["num_nodes"]], dtype=torch.int64, device=device)
    every = torch.empty(world * 3, dtype=torch.int64, device=device)  # flat: gloo takes no (world, 3) output
    dist.all_gather_into_tensor(every, mine)
    every = every.view(world, 3)
    if not (every == mine).all():
        raise SystemExit(f"rank {rank}: ranks disagree on the entry point / index: {every.tolist()}")
    return every


def rank_report(dist, torch, device: str, elapsed: float, queries: int, steps: int, world: int):
    """What the job's record needs to explain itself before an 8-GPU node has run it: how many rank processes the
    collective saw (an all-reduce of ones over the same group the timing's max-over-ranks uses: RCCL on GPUs, gloo in
    the CPU test) and every rank's own rate (an all-gather of the ranks' timed wall times), so a slow or missing rank
    is visible in the line rather than only in `value`."""
    if not dist:
        return 1, [{"rank": 0, "value": queries / elapsed, "ms_per_step": elapsed * 1e3 / steps}]
    one = torch.ones(1, dtype=torch.float64, device=device)
    dist.all_reduce(one)
    mine = torch.tensor([elapsed], dtype=torch.float64, device=device)
    every = torch.empty(world, dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(every, mine)
    per = [{"rank": r, "value": queries / t, "ms_per_step": t * 1e3 / steps} for r, t in enumerate(every.tolist())]
    return int(round(one.item())), per


def peer_access(torch):
    """hipDeviceCanAccessPeer over every pair of the node's GPUs (torch.cuda.can_device_access_peer): the sharded
    placement reads other GPUs' stripes as peer loads (include/shine_gpu.h SHINE_PLACE_SHARDED), so the line records
    whether the node offers them.  None without a GPU (the CPU stub)."""
    if torch is None or not torch.cuda.is_available():
        return {"devices": 0, "can_access": None}
    n = torch.cuda.device_count()
    m = [[True if i == j else bool(torch.cuda.can_device_access_peer(i, j)) for j in range(n)] for i in range(n)]
    return {"devices": n, "can_access": m, "all_pairs": all(all(r) for r in m)}


def attach_sharded_leg(a, world: int, out: dict):
    """The sharded leg after the replica measurement, reported under `sharded`; the replica line is this run's `value`,
    so a failing or hung child (it has never run on more than one physical GPU of this pool) is reported there instead
    of losing the line."""
    if not (a.sharded_leg == "on" or (a.sharded_leg == "auto" and world > 1)):
        return
    try:
        out["sharded"] = sharded_leg(a, world)
    except (SystemExit, Exception) as e:
        log(f"sharded leg failed: {e}")
        out["sharded"] = {"error": str(e)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--nbatches", type=int, default=12, help="distinct query batches per rank (cycled)")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--ef", type=int, default=128)
    p.add_argument("--M", type=int, default=16)
    p.add_argument("--efc", type=int, default=200)
    p.add_argument("--shards", type=int, default=1, help="memory-node dumps the index is spread over")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of the CPU-baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--inflight", type=int, default=4,
                   help="query batches in flight per GPU, each on its own HIP stream (step i runs on stream i %% S), "
                        "so one batch's last queries overlap the next batch's first")
    p.add_argument("--ef-sweep", default="32,48,64,96",
                   help="extra ef values timed in fast mode at N=1 (recall/QPS trade-off; not the headline value)")
    p.add_argument("--mode", choices=["fast", "exact", "both"], default="both",
                   help="search mode(s); the first one measured gives `value` (fast, then exact with 'both')")
    p.add_argument("--cache", default=os.environ.get("SHINE_BENCH_CACHE", "/tmp/shine_bench"))
    p.add_argument("--pmc-json", default=str(ROOT / "profiles" / "r06" / "final" / "sift1m_f32_pmc.json"),
                   help="per-launch HBM bytes of the search kernel measured by rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                        "passes of this bench (tools/pmc.py; tools/gpu_round.sh)")
    p.add_argument("--no-host", action="store_true", help="skip the host-to-host and host-API legs")
    p.add_argument("--rows", choices=["auto", "f32", "u8"], default="f32",
                   help="record storage in HBM for `value` (include/shine_gpu.h SHINE_ELEM_*): f32 as the reference's "
                        "records; auto = the narrowest lossless rows (u8 for SIFT-shaped records, whose components are "
                        "byte values as in the reference's .u8bin inputs); results are bitwise the same")
    p.add_argument("--no-rows-compare", action="store_true",
                   help="skip timing fast mode on the other row storage (byte rows next to f32, or f32 next to bytes)")
    p.add_argument("--builder", choices=["gpu", "cpu"], default="gpu",
                   help="index build: the GPU batch builder (seconds) or the parallel CPU restatement of HNSW::insert")
    p.add_argument("--placement", choices=["replica", "sharded"], default="replica")
    p.add_argument("--slots", type=int, default=0, help="sharded leg: GPU slots (default --gpus)")
    p.add_argument("--cache-frac", type=float, default=0.05,
                   help="sharded leg: share of other stripes cached locally (the reference's default --cache-ratio 5)")
    p.add_argument("--sharded-leg", choices=["auto", "on", "off"], default="auto",
                   help="after the replica measurement, run the cfg-4-shaped sharded leg over the same N GPUs in a child "
                        "process and carry it in the same JSON line (auto: when N > 1)")
    p.add_argument("--sharded-n", type=int, default=10_000_000,
                   help="sharded leg: records of the DEEP-shaped index (10M: every GPU's stripe of vectors and lists is "
                        "~640 MB at 8 GPUs, well above the 256 MiB Infinity Cache)")
    # the launcher hands its flags to the rank processes through the environment: torch.distributed.run's own parser
    # would take bench.py's abbreviations (--n) for its options
    extra = json.loads(os.environ.get("SHINE_BENCH_ARGV", "[]"))
    return p.parse_args(sys.argv[1:] + extra)


def free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def child_json(cmd, env=None, timeout=None):
    """Run a child process (never exec: the parent may have touched the GPU); return its last stdout line parsed as
    JSON.  Its stderr passes through."""
    import subprocess
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env, timeout=timeout)
    if r.returncode != 0:
        raise SystemExit(f"child {cmd[:4]}... exited with {r.returncode}")
    lines = [x for x in r.stdout.splitlines() if x.strip().startswith("{")]
    if not lines:
        raise SystemExit(f"child {cmd[:4]}... printed no JSON line")
    return json.loads(lines[-1])


def forwarded_args(a, drop=("gpus",)):
    """This run's arguments as a command line for a child (bench.py's own flags, `drop` left out)."""
    out = []
    for k, v in vars(a).items():
        if k in drop:
            continue
        flag = "--" + k.replace("_", "-")
        if isinstance(v, bool):
            if v:
                out.append(flag)
        else:
            out += [flag, str(v)]
    return out


def launch(a):
    """`python bench.py --gpus N` (N > 1) without torchrun: this parent never touches the GPU.  It starts
    torch.distributed.run as a child process with N rank processes (one per GPU, rendezvous on 127.0.0.1), which run
    the replica measurement (and, on rank 0, the sharded leg), and relays rank 0's JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve()),
           "--gpus", str(a.gpus)]
    env = dict(os.environ)
    env["SHINE_BENCH_ARGV"] = json.dumps(forwarded_args(a))
    env.setdefault("OMP_NUM_THREADS", str(host_threads()))
    log(f"launching {a.gpus} rank processes: {' '.join(cmd[2:])}")
    line = child_json(cmd, env=env)
    line["launcher"] = "bench.py --gpus N: torch.distributed.run child, one process per GPU"
    print(json.dumps(line), flush=True)


def sharded_leg(a, world: int):
    """The cfg-4-shaped sharded leg over the same GPUs, in a child process (one process drives every GPU slot, so the
    slots' stripes are read over xGMI): a compact summary for the replica line."""
    cmd = [sys.executable, str(Path(__file__).resolve()), "--placement", "sharded", "--gpus", str(world),
           "--slots", str(world), "--n", str(a.sharded_n), "--steps", str(a.steps), "--warmup", str(a.warmup),
           "--batch", str(a.batch), "--nbatches", str(a.nbatches), "--inflight", str(a.inflight), "--mode", "fast",
           "--cache", a.cache, "--cache-frac", str(a.cache_frac)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                           "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID",
                                                           "SHINE_BENCH_ARGV")}
    env["OMP_NUM_THREADS"] = str(max(1, min(host_threads(), 16 * world)))
    t0 = time.time()
    r = child_json(cmd, env=env, timeout=float(os.environ.get("SHINE_SHARDED_LEG_TIMEOUT", "480")))
    keys = ("value", "ms_per_step", "n_gpus", "gpu_slots", "recall_at_10", "search_mode", "scaling", "one_gpu_value",
            "speedup_vs_one_gpu", "reads", "per_slot", "bounds", "config", "data", "stub")
    out = {k: r[k] for k in keys if k in r}
    out["wall_s"] = time.time() - t0
    return out


def main():
    a = parse()
    if a.placement == "sharded":
        return run_sharded(a)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch(a)
    if os.environ.get("SHINE_BENCH_STUB"):
        return stub_rank(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # the in-flight streams first of all streams of the process: distinct hardware queues (hip_streams)
    streams = hip_streams(torch, max(1, a.inflight), local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import shine_amd
    from shine_amd import datasets as D

    key = hashlib.sha1(f"{a.n}-{a.dim}-{a.M}-{a.efc}-{a.shards}-sift_like-v3-{a.builder}".encode()).hexdigest()[:12]
    cache = Path(a.cache) / key
    t0 = time.time()
    base = D.sift_like(a.n, seed=1, d=a.dim)
    log(f"rank {rank}: generated base {base.shape} in {time.time() - t0:.1f}s")
    paths = [cache / "dump" / shine_amd.dump_name(a.M, a.efc, i, a.shards) for i in range(a.shards)]

    def build():
        t0 = time.time()
        if a.builder == "gpu":  # the GPU batch builder on this rank's GPU (include/shine_gpu.h shine_gpu_build)
            with shine_amd.GpuBuild(base, a.M, a.efc, shine_amd.METRIC_L2, seed=1234, gpu=local) as gb:
                dumps = gb.dumps(a.shards)
                st = gb.stats()
            log(f"built index on GPU {local}: {sum(d.size for d in dumps) / 2**20:.0f} MiB in {time.time() - t0:.1f}s "
                f"({st['batches']} batches, GPU build {st['ms_total'] / 1e3:.2f}s)")
            return dumps
        dumps, bdc = shine_amd.build(base, a.M, a.efc, shine_amd.METRIC_L2, a.shards, seed=1234,
                                     threads=host_threads())
        log(f"built index: {sum(d.size for d in dumps) / 2**20:.0f} MiB in {time.time() - t0:.1f}s "
            f"({host_threads()} threads, {bdc} distcomps)")
        return dumps

    prepare_dumps(paths, rank, dist, build)
    elem = {"auto": shine_amd.ELEM_AUTO, "f32": shine_amd.ELEM_F32, "u8": shine_amd.ELEM_U8}[a.rows]
    idx = shine_amd.Index.open(paths, a.dim, a.M, shine_amd.METRIC_L2, elem=elem, gpus=[local])
    info = idx.info()
    rows = ROW_NAMES[info["elem"]]
    log(f"rank {rank}: index on GPU {local}: {info['num_nodes']} nodes, max level {info['max_level']}, "
        f"{info['device_bytes'] / 2**20:.0f} MiB ({rows} rows); device {info['cus']} CUs, {info['lds_per_cu']} B LDS per CU")
    if dist:
        check_same_index(dist, torch, info, world, rank, f"cuda:{local}")

    # queries: rank r takes ids ≡ r (mod G) of a common pool (read_data.hh:57-58)
    nq_rank = a.batch * a.nbatches
    pool = D.sift_like(nq_rank * world, seed=2, d=a.dim)
    q = rank_queries(pool, rank, world, nq_rank)
    qd = torch.from_numpy(q).cuda()
    ids = torch.empty((a.nbatches, a.batch, a.k), dtype=torch.int32, device="cuda")
    dists = torch.empty((a.nbatches, a.batch, a.k), dtype=torch.float32, device="cuda")
    qs = torch.zeros((a.nbatches, a.batch, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    # real streams (the C ABI reads a NULL stream as "the handle's own stream"); the index keeps device scratch per
    # stream, so batches on different streams run concurrently
    if a.nbatches < a.inflight:
        raise SystemExit("--nbatches must be >= --inflight (batches in flight write distinct output buffers)")
    torch.cuda.set_stream(streams[0])

    def step(i, rec=None, ef=None, ix=None):
        b = i % a.nbatches
        stream = streams[i % len(streams)]
        if rec is not None:
            rec[0].record(stream)
        (ix or idx).knn_device(qd[b * a.batch:(b + 1) * a.batch].data_ptr(), a.batch, a.k, ef or a.ef, ids[b].data_ptr(),
                       dists[b].data_ptr(), qs[b].data_ptr(), stream=stream.cuda_stream)
        if rec is not None:
            rec[1].record(stream)

    gt = ground_truth(torch, base, q, a.k, 0)

    def run_mode(mode, ix=None, ef=None):
        """Validation pass over every batch (status, recall, algorithmic bytes), warmup, then exactly K timed
        steps between barriers; returns the measurements."""
        ix = ix or idx
        ix.set_search_mode(mode)
        for i in range(a.nbatches):
            step(i, ix=ix, ef=ef)
        torch.cuda.synchronize()
        qs_h = qs.cpu().numpy().view(np.uint32).reshape(-1, shine_amd.QS_WORDS).copy()
        n_bad = int((qs_h[:, 6] != 0).sum())
        if n_bad:
            raise SystemExit(f"{n_bad} queries did not complete (status {np.unique(qs_h[:, 6])})")
        bq_batch = [ix.algorithmic_bytes(qs_h[b * a.batch:(b + 1) * a.batch]) for b in range(a.nbatches)]
        res = ids.cpu().numpy().view(np.uint32).reshape(-1, a.k).copy()
        res_d = dists.cpu().numpy().copy()
        recall = D.recall_at_k(res, gt, a.k)
        log(f"rank {rank}: mode {mode}: recall@{a.k} = {recall:.4f} over {nq_rank} queries; mean distcomps "
            f"{qs_h[:, 0].mean():.0f}, lists L0 {qs_h[:, 4].mean():.1f}")
        for i in range(a.warmup):
            step(i, ix=ix, ef=ef)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i, evs[i], ix=ix, ef=ef)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        elapsed = max_over_ranks(t1 - t0, dist, "cuda")
        elapsed_rank = t1 - t0
        kern_ms = [s.elapsed_time(e) for s, e in evs]
        span_ms = max(evs[0][0].elapsed_time(e) for _, e in evs)  # first launch's start to the last one's end
        bytes_steps = [bq_batch[(a.warmup + i) % a.nbatches] for i in range(a.steps)]
        return dict(elapsed=elapsed, elapsed_rank=elapsed_rank, kern_ms=kern_ms, span_ms=span_ms,
                    bytes_steps=bytes_steps, recall=recall, qs=qs_h, ids=res, dists=res_d)

    def host_legs(mode, ref_ids):
        """SURVEY §8d's query phase, host to host, K steps between barriers, batches in flight as above:
        zero copy (`value_host_to_host`): queries in pinned host memory, the kernels read them and write ids and
        distances into pinned host memory over PCIe (the device address space maps it); copy engine
        (`value_host_to_host_copies`): pinned H2D → knn → D2H on the step's stream; then the synchronous C-ABI host
        call (shine_knn_batch, zero-copy staging inside the library), one batch at a time.  The zero-copy answers
        are checked against the HBM-resident run's."""
        idx.set_search_mode(mode)
        q_host = torch.from_numpy(q).pin_memory()
        ids_host = torch.empty((a.nbatches, a.batch, a.k), dtype=torch.int32).pin_memory()
        d_host = torch.empty((a.nbatches, a.batch, a.k), dtype=torch.float32).pin_memory()
        qbuf = [torch.empty((a.batch, a.dim), dtype=torch.float32, device="cuda") for _ in streams]

        def hstep(i, copies):
            b, si = i % a.nbatches, i % len(streams)
            st = streams[si]
            if not copies:
                idx.knn_device(q_host[b * a.batch:(b + 1) * a.batch].data_ptr(), a.batch, a.k, a.ef,
                               ids_host[b].data_ptr(), d_host[b].data_ptr(), qs[b].data_ptr(), stream=st.cuda_stream)
                return
            with torch.cuda.stream(st):
                qbuf[si].copy_(q_host[b * a.batch:(b + 1) * a.batch], non_blocking=True)
                idx.knn_device(qbuf[si].data_ptr(), a.batch, a.k, a.ef, ids[b].data_ptr(), dists[b].data_ptr(),
                               qs[b].data_ptr(), stream=st.cuda_stream)
                ids_host[b].copy_(ids[b], non_blocking=True)
                d_host[b].copy_(dists[b], non_blocking=True)

        def timed(copies):
            for i in range(a.nbatches):  # every batch once: the answers checked below
                hstep(i, copies)
            torch.cuda.synchronize()
            got = ids_host.numpy().view(np.uint32).reshape(-1, a.k).copy()
            for i in range(a.warmup):
                hstep(i, copies)
            torch.cuda.synchronize()
            if dist:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                hstep(a.warmup + i, copies)
            torch.cuda.synchronize()
            return max_over_ranks(time.perf_counter() - t0, dist, "cuda"), got

        el, got = timed(False)
        out = {"value_host_to_host": a.steps * a.batch * world / el, "ms_per_step_host_to_host": el * 1e3 / a.steps,
               "host_to_host_same_ids_as_device": bool(ref_ids is not None and (got == ref_ids).all()),
               "recall_at_10_host_to_host": D.recall_at_k(got, gt, a.k)}
        el, _ = timed(True)
        out["value_host_to_host_copies"] = a.steps * a.batch * world / el
        # the drop-in host API (shine_knn_batch: host arrays in, host arrays out, returns when the results are there),
        # as the compute-node façade calls it: the rank's whole query set per call, which the library runs as 1,024-query
        # chunks kept in flight on four streams (capi.cc knn_host; compute_node.cc:354-386 keeps T x C queries in
        # flight), repeated to at least K batches' worth of queries
        calls = max(1, -(-a.steps // a.nbatches))
        api_ids = idx.knn(q, a.k, a.ef).ids
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(calls):
            idx.knn(q, a.k, a.ef)
        el = max_over_ranks(time.perf_counter() - t0, dist, "cuda")
        out["value_host_api_sync"] = calls * q.shape[0] * world / el
        # the same calls through shine_knn_batch_async, the next call enqueued before the previous one is waited for
        # (two in flight: the GPU does not drain between calls), at least three calls
        acalls = max(3, calls)
        async_ids = idx.knn_async(q, a.k, a.ef).wait().ids
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        pending = []
        for _ in range(acalls):
            pending.append(idx.knn_async(q, a.k, a.ef))
            if len(pending) >= 2:
                pending.pop(0).wait()
        for r in pending:
            r.wait()
        el = max_over_ranks(time.perf_counter() - t0, dist, "cuda")
        out["value_host_api"] = acalls * q.shape[0] * world / el
        out["ms_per_step_host_api"] = el * 1e3 / (acalls * a.nbatches)
        out["host_api_calls"] = {"calls": acalls, "queries_per_call": int(q.shape[0]), "calls_in_flight": 2,
                                 "entry": "shine_knn_batch_async + shine_wait",
                                 "same_ids_as_device": bool(ref_ids is not None and (api_ids == ref_ids).all()),
                                 "async_same_ids_as_sync": bool((async_ids == api_ids).all()),
                                 "sync_calls": calls}
        # the same API one batch per call (nothing in flight between calls: the round-4 leg)
        steps_api = max(1, min(a.steps, 20))
        t0 = time.perf_counter()
        for i in range(steps_api):
            b = i % a.nbatches
            idx.knn(q[b * a.batch:(b + 1) * a.batch], a.k, a.ef)
        el = max_over_ranks(time.perf_counter() - t0, dist, "cuda")
        out["value_host_api_per_batch"] = steps_api * a.batch * world / el
        log(f"host legs: host-to-host zero copy {out['value_host_to_host'] / 1e6:.2f}M QPS (same ids as on HBM: "
            f"{out['host_to_host_same_ids_as_device']}), copy engine {out['value_host_to_host_copies'] / 1e6:.2f}M, "
            f"shine_knn_batch {out['value_host_api'] / 1e6:.2f}M QPS")
        return out

    if a.nbatches % max(1, a.inflight) != 0:
        raise SystemExit("--nbatches must be a multiple of --inflight (a batch's buffers stay on one stream)")
    modes = ["fast", "exact"] if a.mode == "both" else [a.mode]
    runs = {m: run_mode(shine_amd.MODE_FAST if m == "fast" else shine_amd.MODE_EXACT) for m in modes}
    other_rows = None
    if "fast" in runs and not a.no_rows_compare:
        # the same search on the other row storage: f32 rows (4 B per component) next to byte rows, or the narrowest
        # lossless rows next to f32; same results bit for bit, different bytes per distance
        oelem = shine_amd.ELEM_F32 if rows != "f32" else shine_amd.ELEM_AUTO
        with shine_amd.Index.open(paths, a.dim, a.M, shine_amd.METRIC_L2, elem=oelem, gpus=[local]) as io:
            orows = ROW_NAMES[io.info()["elem"]]
            ro = run_mode(shine_amd.MODE_FAST, io) if orows != rows else None
        if ro is not None:
            fr = runs["fast"]
            other_rows = {"rows": orows, "value": a.steps * a.batch * world / ro["elapsed"],
                          "ms_per_step": ro["elapsed"] * 1e3 / a.steps, "avg_launch_ms": float(np.mean(ro["kern_ms"])),
                          "recall_at_10": ro["recall"],
                          "roofline_frac": sum(ro["bytes_steps"]) / (ro["span_ms"] / 1e3) / 1e9 / HBM_PEAK_GBPS,
                          "algorithmic_bytes_per_launch": float(np.mean(ro["bytes_steps"])),
                          "kernel": f"search_fast_kernel<128,L2,{orows},R=2,P=2>",
                          "same_ids_dists_counters": bool(
                              (ro["ids"] == fr["ids"]).all() and (ro["dists"].view(np.uint32) == fr["dists"].view(np.uint32)).all()
                              and (ro["qs"][:, :8] == fr["qs"][:, :8]).all())}
            log(f"{orows} rows: {other_rows['value'] / 1e6:.2f}M QPS, frac {other_rows['roofline_frac']:.3f}, identical "
                f"results: {other_rows['same_ids_dists_counters']}")
    host = None if a.no_host else host_legs(shine_amd.MODE_FAST if modes[0] == "fast" else shine_amd.MODE_EXACT,
                                            runs[modes[0]]["ids"])
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
            qs_e = qs.cpu().numpy().view(np.uint32).reshape(-1, shine_amd.QS_WORDS)
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

    best = max((x for x in sweep if x["recall_at_10"] >= 0.95), key=lambda x: x["value"], default=None)
    if other_rows is not None and best is not None and best["ef"] != a.ef:
        # the other rows at the metric's bar too (the fastest swept ef with recall@10 >= 0.95)
        with shine_amd.Index.open(paths, a.dim, a.M, shine_amd.METRIC_L2, elem=oelem, gpus=[local]) as io:
            rb = run_mode(shine_amd.MODE_FAST, io, ef=best["ef"])
        other_rows["at_best_ef"] = {"ef": best["ef"], "value": a.steps * a.batch * world / rb["elapsed"],
                                    "recall_at_10": rb["recall"], "same_recall_as_f32_rows": rb["recall"] == best["recall_at_10"]}
        log(f"{other_rows['rows']} rows at ef={best['ef']}: {other_rows['at_best_ef']['value'] / 1e6:.2f}M QPS")

    traffic, traffic_src = None, None
    if a.pmc_json and Path(a.pmc_json).exists():
        pmc = json.loads(Path(a.pmc_json).read_text())
        want = f"void shine::(anonymous namespace)::search_fast_kernel<128, 0, {KERNEL_TYPE[rows]}, 2,"
        if any(k.startswith(want) for k in pmc.get("kernels", [])):
            traffic = pmc.get("hbm_bytes_per_launch")
            traffic_src = str(Path(a.pmc_json).relative_to(ROOT)) if Path(a.pmc_json).is_relative_to(ROOT) else a.pmc_json

    ranks_seen, per_rank = rank_report(dist, torch, "cuda", head["elapsed_rank"], a.steps * a.batch, a.steps, world)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(paths, q, a, gt, runs["exact"]["ids"] if "exact" in runs else None)

    if rank == 0:
        total_q = a.steps * a.batch * world
        out = {
            "metric": "QPS at recall@10>=0.95, SIFT1M d=128 batch=1024",
            "value": total_q / elapsed,
            "unit": "queries/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "per_rank": per_rank,
            "peer_access": peer_access(torch),
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "rows": rows,
            "data": "synthetic SIFT-shaped (byte-valued f32 records, 1M x 128, as SIFT's .u8bin), random-seeded; "
                    f"index built in-run ({'GPU batch builder' if a.builder == 'gpu' else 'CPU builder'})",
            "recall_at_10": recall,
            **(host or {}),
            "search_mode": modes[0],
            "modes": mode_report,
            "other_rows": other_rows,
            "ef_sweep": sweep or None,
            "best_at_recall_0.95": best,
            "config": {"workload": "SIFT1M-shaped L2 knn, M=16 efC=200 ef=128 k=10", "n": a.n, "dim": a.dim,
                       "global_batch": a.batch * world, "batch_per_gpu": a.batch, "M": a.M, "efc": a.efc,
                       "ef": a.ef, "k": a.k, "shards": a.shards, "parallelism": f"replica{world}",
                       "batches_in_flight": len(streams), "rows": rows,
                       # the GPU batch builder's graph is not the sequential insert's: at this size its recall@10 is
                       # within 1e-4 of the CPU builder's (profiles/r04/cmp1m_gpu_vs_cpu_build.jsonl); --builder cpu
                       # runs the restatement of HNSW::insert instead
                       "builder": "gpu batch builder (shine_gpu_build)" if a.builder == "gpu" else
                                  "CPU restatement of HNSW::insert (shine_build)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": (f"search_fast_kernel<128,L2,{rows},R=2,P=2>" if modes[0] == "fast"
                                    else f"search_kernel<128,L2,{rows},0>"), "avg_launch_ms": avg_launch_ms,
                         "span_ms_per_launch": span_ms / a.steps, "batches_in_flight": len(streams),
                         "achieved_basis": "algorithmic bytes of the K timed launches / their GPU span (first "
                                           "launch start to last launch end, HIP events on the launch streams)",
                         "algorithmic_bytes_per_launch": float(np.mean(bytes_steps)),
                         "mean_distcomps_per_query": float(qs_h[:, 0].mean())},
            "cpu_baseline": cpu,
            "hw_queues": HW_QUEUES or "HIP default (4)",
            # provenance of the measured library: its source hash must equal the tree's (a stale .so is visible here)
            "build_id": shine_amd._lib.build_id(),
            "tree_source_hash": shine_amd._lib.source_hash(),
        }
    idx.close()
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        del qd, ids, dists, qs
        torch.cuda.empty_cache()
        attach_sharded_leg(a, world, out)
        print(json.dumps(out), flush=True)


def stub_rank(a):
    """SHINE_BENCH_STUB=1 (CPU tests of the launcher): each rank joins a gloo group instead of doing GPU work; rank 0
    counts the ranks with an all-reduce, runs the sharded-leg child (itself a stub) and prints a line of the real
    line's shape."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        # the same entry-point check the GPU ranks run, over gloo, on a stand-in index description
        check_same_index(dist, torch, {"entry_uid": 7, "max_level": 3, "num_nodes": 1000}, world, rank, "cpu")
    # the same per-rank report as the GPU ranks, on a stand-in timing (rank r "took" 1 + r/10 s)
    seen, per_rank = rank_report(dist, torch, "cpu", 1.0 + rank / 10, a.steps * a.batch, a.steps, world)
    if dist:
        dist.destroy_process_group()
    if rank != 0:
        return
    out = {"metric": "QPS at recall@10>=0.95, SIFT1M d=128 batch=1024", "value": 0.0, "unit": "queries/s",
           "n_gpus": world, "ranks_seen": seen, "per_rank": per_rank, "peer_access": peer_access(None), "stub": True,
           "scaling": "weak", "config": {"parallelism": f"replica{world}"}}
    attach_sharded_leg(a, world, out)
    print(json.dumps(out), flush=True)


def sharded_plan(slots: int, ndev: int, batch: int, nbatches: int):
    """GPU of every slot of the sharded leg (slot s on device s % ndev, so N slots over N devices is one slot per
    GPU and more slots than devices repeat them) and the query rows each slot answers in every batch: the
    compute-node split by query id, id % slots (read_data.hh:57-58)."""
    if slots < 1 or ndev < 1:
        raise SystemExit("--placement sharded needs at least one slot and one GPU")
    gpus = [s % ndev for s in range(slots)]
    ids = [np.arange(b * batch, (b + 1) * batch) for b in range(nbatches)]
    rows = [[ids[b][ids[b] % slots == s] for s in range(slots)] for b in range(nbatches)]
    return gpus, rows


def run_sharded(a):
    """cfg-4-shaped sharded leg: one process drives S GPU slots of one index in the sharded placement
    (include/shine_gpu.h SHINE_PLACE_SHARDED): memory node m lives on slot m % S only, every slot reads the others'
    stripes through its own virtual view (xGMI when the slots are distinct GPUs), queries split id % S.  Reports
    QPS, recall, the share of the algorithmic bytes that left the answering slot's stripe (qstats words 8-11) and the
    xGMI bound that share implies (7 links x 153 GB/s inbound per GPU)."""
    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("--placement sharded runs as one process driving every GPU slot (not under torchrun)")
    if os.environ.get("SHINE_BENCH_STUB"):
        if os.environ.get("SHINE_BENCH_STUB_FAIL_SHARDED"):  # CPU test: a sharded child that fails
            raise SystemExit(3)
        S = a.slots or a.gpus
        print(json.dumps({"value": 0.0, "n_gpus": a.gpus, "gpu_slots": S, "stub": True,
                          "per_slot": [{"slot": s, "gpu": s % max(1, a.gpus), "span_ms_per_step": None,
                                        "reads": None} for s in range(S)]}), flush=True)
        return
    import torch
    import shine_amd
    from shine_amd import datasets as D
    ndev = torch.cuda.device_count()
    S = a.slots or a.gpus
    # every slot answers a.batch queries per step (global batch a.batch x S, split id % S): per-GPU work is fixed
    gpus, rows = sharded_plan(S, ndev, a.batch * S, a.nbatches)
    phys = len(set(gpus))
    # the in-flight streams of every slot, created first in the process through HIP (hip_streams): torch's stream
    # pool can put two batches on one hardware queue (this leg read 3.07 M QPS on one slot of one GPU where the same
    # layout measures 5.36 M on reserved streams, profiles/r04/layout_probe.jsonl)
    per_dev: dict = {}
    for s in range(S):
        per_dev.setdefault(gpus[s], []).append(s)
    slot_streams = {}
    for d, slots_d in per_dev.items():
        made = hip_streams(torch, max(1, a.inflight) * len(slots_d), d)
        for j, s in enumerate(slots_d):
            slot_streams[s] = made[j * max(1, a.inflight):(j + 1) * max(1, a.inflight)]
    dim, M, efc, ef, shards = 96, 16, 200, 128, 8
    # the index is built on GPU 0 by the GPU batch builder (10M records in seconds) and laid out over the slots as its
    # 8 memory-node dumps would be (shine_gpu_build_open_ex), without writing or parsing them
    base_t = D.generate_device("deep_like", a.n, seed=1, d=dim)
    t0 = time.time()
    gb = shine_amd.GpuBuild(base_t.data_ptr(), M, efc, shine_amd.METRIC_L2, seed=1234, n=a.n, dim=dim)
    log(f"built the sharded leg's index ({a.n} x {dim}) on GPU 0 in {time.time() - t0:.1f}s")
    t0 = time.time()
    idx = gb.open_ex(shards, gpus=gpus, placement="sharded", cache=a.cache_frac)
    info = idx.info()
    log(f"sharded index: {info['num_nodes']} nodes over {S} slots ({phys} GPUs), id space {info['id_space']}, "
        f"{info['device_bytes'] / 2**20:.0f} MiB per GPU, cache fraction {info['cache_fraction']:.3f}, laid out in "
        f"{time.time() - t0:.1f}s")
    nb, B, k = a.nbatches, a.batch * S, a.k
    q_t = D.generate_device("deep_like", B * nb, seed=2, d=dim)
    gt = D.ground_truth_device(base_t, q_t, k, 0)
    q = q_t.cpu().numpy()
    del base_t, q_t
    torch.cuda.empty_cache()
    qd, ids, qs, streams = [], [], [], []
    for s in range(S):
        dev = torch.device("cuda", gpus[s])
        qd.append([torch.from_numpy(np.ascontiguousarray(q[rows[b][s]])).to(dev) for b in range(nb)])
        ids.append([torch.empty((len(rows[b][s]), k), dtype=torch.int32, device=dev) for b in range(nb)])
        qs.append([torch.zeros((len(rows[b][s]), shine_amd.QS_WORDS), dtype=torch.int32, device=dev)
                   for b in range(nb)])
        streams.append(slot_streams[s])

    def step(i, evs=None):
        b = i % nb
        for s in range(S):
            n = len(rows[b][s])
            if n:
                st = streams[s][i % len(streams[s])]
                if evs is not None:
                    evs[s].append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                    with torch.cuda.device(gpus[s]):
                        evs[s][-1][0].record(st)
                idx.knn_device(qd[s][b].data_ptr(), n, k, ef, ids[s][b].data_ptr(), None, qs[s][b].data_ptr(),
                               stream=st.cuda_stream, gpu_slot=s)
                if evs is not None:
                    with torch.cuda.device(gpus[s]):
                        evs[s][-1][1].record(st)

    def sync():
        for d in sorted(set(gpus)):
            torch.cuda.synchronize(d)

    lines = []
    for mode_name, mode in (("fast", shine_amd.MODE_FAST), ("exact", shine_amd.MODE_EXACT)):
        if a.mode != "both" and a.mode != mode_name:
            continue
        idx.set_search_mode(mode)
        for i in range(nb):
            step(i)
        sync()
        res = np.zeros((B * nb, k), np.uint32)
        st = np.zeros((B * nb, shine_amd.QS_WORDS), np.uint32)
        for b in range(nb):
            for s in range(S):
                res[rows[b][s]] = ids[s][b].cpu().numpy().view(np.uint32)
                st[rows[b][s]] = qs[s][b].cpu().numpy().view(np.uint32)
        if (st[:, 6] != 0).any():
            raise SystemExit(f"{int((st[:, 6] != 0).sum())} queries failed")
        recall = D.recall_at_k(res, gt, k)
        for i in range(a.warmup):
            step(i)
        sync()
        evs = [[] for _ in range(S)]
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i, evs)
        sync()
        el = time.perf_counter() - t0
        # every slot's own GPU span over the K steps (its first launch's start to its last launch's end, HIP events on
        # its streams) and its read classes (qstats words 8-11 per query it answered: vector / list reads over xGMI,
        # vector / list reads served by its local copies)
        per_slot = []
        for s in range(S):
            span = max(evs[s][0][0].elapsed_time(e) for _, e in evs[s]) if evs[s] else None
            mine = np.concatenate([np.asarray(rows[b][s], dtype=np.int64) for b in range(nb)])
            cls = st[mine][:, 8:12].astype(np.float64).mean(0) if mine.size else np.zeros(4)
            per_slot.append({"slot": s, "gpu": gpus[s], "span_ms_per_step": span / a.steps if span else None,
                             "queries_per_step": int(np.mean([len(rows[b][s]) for b in range(nb)])),
                             "reads": {"xgmi_vec_per_query": cls[0], "xgmi_list_per_query": cls[1],
                                       "cached_vec_per_query": cls[2], "cached_list_per_query": cls[3]}})
        algo = idx.algorithmic_bytes(st) / st.shape[0]
        remote = (st[:, 8].astype(np.float64) * dim * 4 + st[:, 9].astype(np.float64) * 4 * 2 * M).mean()
        vec_hits, vec_remote = int(st[:, 10].sum()), int(st[:, 8].sum())
        hits, misses = int(st[:, 10:12].sum()), int(st[:, 8:10].sum())
        node_reads = int(st[:, 0].sum())  # every distance computation reads one record (rdma::read_node)
        qps = a.steps * B / el
        one = (one_gpu_rate(a, torch, shine_amd, gb, dim, M, ef, k, q, rows, mode, slot_streams[per_dev[0][0]])
               if mode_name == "fast" and 0 in per_dev else None)
        xgmi_in = 7 * 153e9
        line = {
            "metric": "QPS at recall@10, cfg4-shaped sharded index (DEEP-like 96-d L2, 8 memory-node dumps)",
            "value": qps, "unit": "queries/s", "n_gpus": phys, "gpu_slots": S, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": el * 1e3 / a.steps, "higher_is_better": True, "vs_baseline": None,
            "scaling": "weak in queries (a.batch per slot per step) over one fixed index",
            "one_gpu_value": one, "speedup_vs_one_gpu": (qps / one) if one else None,
            "dtype": "f32", "search_mode": mode_name, "recall_at_10": recall,
            "data": f"synthetic DEEP-shaped (L2-normalised f32, {a.n} x 96, GPU-generated; N reduced from 100M), index "
                    f"built in-run on GPU 0 (shine_gpu_build)",
            "config": {"workload": "cfg4-shaped sharded knn, M=16 efC=200 ef=128 k=10", "n": a.n, "dim": dim,
                       "M": M, "efc": efc, "ef": ef, "k": k, "shards": shards, "batch": B, "batch_per_slot": a.batch,
                       "placement": "sharded", "gpus": gpus, "cache_fraction": info["cache_fraction"],
                       "batches_in_flight": max(1, a.inflight)},
            "reads": {"algorithmic_bytes_per_query": algo, "off_stripe_bytes_per_query": remote,
                      "off_stripe_share": remote / algo,
                      # statistics.hh:171-173: hits over every record lookup (the reference reads every record
                      # remotely, so every node read is a cache lookup there)
                      "cache_hit_rate": vec_hits / max(1, node_reads),
                      "off_stripe_hit_rate": vec_hits / max(1, vec_hits + vec_remote),
                      "node_reads": node_reads, "cache_hits": vec_hits, "cache_misses": node_reads - vec_hits,
                      "off_stripe_record_hits": hits, "off_stripe_record_misses": misses},
            "per_slot": per_slot,
            "bounds": {"hbm_qps": phys * HBM_PEAK_GBPS * 1e9 / algo,
                       "xgmi_qps": (phys * xgmi_in / remote) if phys > 1 and remote > 0 else None,
                       "note": "xgmi_qps: every GPU's off-stripe reads at 7 x 153 GB/s inbound; with repeated slots "
                               "on one GPU all reads are local HBM and only the accounting is exercised"},
        }
        log(json.dumps(line))
        lines.append(line)
    idx.close()
    gb.close()
    print(json.dumps(lines[0]), flush=True)


def one_gpu_rate(a, torch, shine_amd, gb, dim, M, ef, k, q, rows, mode, streams):
    """The same index as a replica on GPU 0 (the build's own arrays), the same global batches (each slot's share one
    launch, in flight on rotating streams — GPU 0's first slot's reserved streams): the one-GPU rate the sharded leg's
    speedup is quoted against."""
    nb, S = len(rows), len(rows[0])
    with gb.open_ex(1, gpus=[0]) as ix:
        ix.set_search_mode(mode)
        with torch.cuda.device(0):
            qd = [[torch.from_numpy(np.ascontiguousarray(q[rows[b][s]])).cuda() for s in range(S)] for b in range(nb)]
            ids = [[torch.empty((len(rows[b][s]), k), dtype=torch.int32, device="cuda") for s in range(S)]
                   for b in range(nb)]
        n_launch = [0]

        def step(i):
            b = i % nb
            for s in range(S):
                n = len(rows[b][s])
                if n:
                    ix.knn_device(qd[b][s].data_ptr(), n, k, ef, ids[b][s].data_ptr(), None, None,
                                  stream=streams[n_launch[0] % len(streams)].cuda_stream)
                    n_launch[0] += 1

        for i in range(nb + a.warmup):
            step(i)
        torch.cuda.synchronize(0)
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(a.warmup + i)
        torch.cuda.synchronize(0)
        el = time.perf_counter() - t0
    B = sum(len(r) for r in rows[0])
    return a.steps * B / el


def ground_truth(torch, base, q, k, metric):
    """Exact top-k on the GPU in float64 (no reduced-precision GEMM path can reorder near neighbours)."""
    bt = torch.from_numpy(base).cuda().double()
    bn = (bt * bt).sum(1)
    qd = torch.from_numpy(q).cuda().double()
    out = []
    for s in range(0, q.shape[0], 256):
        qq = qd[s:s + 256]
        ip = qq @ bt.T
        dd = (qq * qq).sum(1)[:, None] + bn[None, :] - 2.0 * ip if metric == 0 else 1.0 - ip
        out.append(torch.topk(dd, k, largest=False).indices.cpu().numpy())
    del bt, bn, qd
    torch.cuda.empty_cache()
    return np.concatenate(out)


def host_cpu_info():
    """nproc and lscpu's socket / core counts of the host that runs the CPU baseline."""
    import subprocess
    info = {"nproc": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            key, _, val = line.partition(":")
            key, val = key.strip(), val.strip()
            if key in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)"):
                info[{"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                      "Thread(s) per core": "threads_per_core", "CPU(s)": "cpus"}[key]] = val
    except Exception as e:  # lscpu absent: report what os gives
        info["lscpu_error"] = str(e)
    return info


def native_oracle():
    """Build the oracle with the reference's flags for THIS host (-march=native must target the CPU being timed).
    Returns True if the native build is usable, else the portable checker build is timed instead."""
    import subprocess
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    try:
        subprocess.run(["make", "-s", "-B", "-C", str(ROOT / "oracle"), "native"], check=True, capture_output=True,
                       timeout=300)
        return O.NATIVE_PATH.exists()
    except Exception as e:
        log(f"native oracle build failed ({e}); timing the portable build")
        return False


def granted_cpus(n: int):
    """The first n CPUs of this process's affinity mask (the CPUs the box grants this job)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except Exception:
        cpus = list(range(os.cpu_count() or 1))
    return cpus[:max(1, n)]


def fp_order_probe(O, native, dumps, dim, M, metric, q, k, ef, threads, cpus, gpu_ids=None):
    """The -ffast-math question: the oracle built with the reference's flags against the portable checker
    build (explicit FMA chain, fixed left-to-right horizontal sum) on the same queries and dump."""
    chk = O.OracleIndex(dumps, dim, M, metric)
    ci, cd, _ = chk.knn(q, k, ef, threads=threads, cpus=cpus)
    chk.close()
    out = {"queries": int(q.shape[0])}
    if native:
        nat = O.OracleIndex(dumps, dim, M, metric, native=True)
        ni, nd, _ = nat.knn(q, k, ef, threads=threads, cpus=cpus)
        nat.close()
        out["native_same_ids"] = float((ni == ci).all(1).mean())
        out["native_same_id_sets"] = float((np.sort(ni, 1) == np.sort(ci, 1)).all(1).mean())
        same = ni == ci  # positions holding the same record in both builds
        out["native_dist_bitwise_rate"] = float((nd.view(np.uint32) == cd.view(np.uint32))[same].mean())
        ulp = np.abs(nd.view(np.int32).astype(np.int64) - cd.view(np.int32).astype(np.int64))[same]
        out["native_max_ulp_diff"] = int(ulp.max()) if ulp.size else 0
        out["native_max_abs_dist_diff"] = float(np.abs(nd.astype(np.float64) - cd)[same].max()) if same.any() else 0.0
    if gpu_ids is not None:
        out["checker_same_ids_as_gpu_exact"] = float((gpu_ids[:q.shape[0]] == ci).all(1).mean())
    return out, ci


def cpu_baseline(paths, q, a, gt, gpu_exact_ids=None):
    """The oracle (C++ restatement of the reference's knn) on this host's cores, same dump, same queries: built with
    the reference's flags (-O3 -march=native -ffast-math -mavx2) for this host, one worker per granted CPU, each
    pinned to its CPU (compute_node.cc:362-380).  Also reported: its recall on the sample, and the fp-order probe —
    the native build against the portable checker build on this sample and on a float-valued DEEP-shaped
    inner-product index, where -ffast-math could reorder the distance sums."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O
    from shine_amd import datasets as D
    import shine_amd
    native = native_oracle()
    dumps = [np.fromfile(p, dtype=np.uint8) for p in paths]
    th = host_threads()
    cpus = granted_cpus(th)
    th = len(cpus)
    I = O.OracleIndex(dumps, a.dim, a.M, 0, native=native)
    n = min(q.shape[0], 512)
    t0 = time.perf_counter()
    I.knn(q[:n], a.k, a.ef, threads=th, cpus=cpus)
    probe = time.perf_counter() - t0
    reps = max(1, int(a.cpu_seconds / max(probe, 1e-3)))
    t0 = time.perf_counter()
    done, got = 0, {}
    for r in range(reps):
        s = (r * n) % max(1, q.shape[0] - n + 1)
        ids, _, _ = I.knn(q[s:s + n], a.k, a.ef, threads=th, cpus=cpus)
        done += n
        got.setdefault(s, ids)
    el = time.perf_counter() - t0
    I.close()
    rows = sorted(got)
    cpu_ids = np.concatenate([got[s] for s in rows])
    cpu_gt = np.concatenate([gt[s:s + n] for s in rows])
    recall = D.recall_at_k(cpu_ids, cpu_gt, a.k)
    probe_sift, _ = fp_order_probe(O, native, dumps, a.dim, a.M, 0, q[:n], a.k, a.ef, th, cpus,
                                   gpu_ids=gpu_exact_ids)
    # float data: a DEEP-shaped inner-product index (cfg 3's metric), 20K records, 1,024 queries at ef = 256
    base_f = D.deep_like(20_000, seed=31, d=96)
    q_f = D.deep_like(1024, seed=32, d=96)
    dumps_f, _ = shine_amd.build(base_f, 16, 100, shine_amd.METRIC_IP, 1, seed=1234, threads=th)
    probe_deep, _ = fp_order_probe(O, native, dumps_f, 96, 16, 1, q_f, a.k, 256, th, cpus)
    hw = host_cpu_info()
    log(f"cpu baseline: {done} queries in {el:.1f}s on {th} pinned threads, recall {recall:.4f} ({hw}); fp-order "
        f"probe sift {probe_sift}, deep-ip {probe_deep}")
    return {"value": done / el, "unit": "queries/s", "cores": th, "kind": "port",
            "flags": O.NATIVE_FLAGS if native else "-O3 -march=x86-64-v3 -ffp-contract=off (portable checker build)",
            "host": hw, "pinned": True, "cpus": cpus, "recall_at_10": recall,
            "fp_order_probe": {"sift_sample": probe_sift, "deep_ip_20k": probe_deep},
            "label": "reference-equivalent CPU path (restated), not the RDMA deployment",
            "sample": f"{done} queries (batches of {n} from the bench's query set, k={a.k}, ef={a.ef}) on the "
                      f"same dump, {th} worker threads pinned one per granted CPU, ~{a.cpu_seconds:.0f}s"}


if __name__ == "__main__":
    main()
