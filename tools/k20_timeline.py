#!/usr/bin/env python3
"""Where the driver's 20-step bench run loses to the 200-step one (6.00 M against 6.65 M QPS in round 5): the bench's
timed loop (four batches in flight on reserved streams, fast mode, SIFT-shaped 1M x 128, GPU-built) repeated, with per
step the host time at which its enqueue returned and the GPU events around it.  Per repetition: wall time, the event
span (first step's start to the last step's end), and the step timeline relative to the first start — the ramp (how
long until four batches run), the steady spacing and the drain (the last batch's end after the others').

Usage: python tools/k20_timeline.py [--steps 20] [--reps 5] [--out gpurun_out/k20_timeline.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
from bench import log  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--ef", type=int, default=128)
    p.add_argument("--mode", default="fast", help="modes run in turn on one handle, e.g. fast,exact (as bench.py does)")
    p.add_argument("--inflight", type=int, default=4)
    p.add_argument("--envs", default="", help="';'-separated variants (KEY=VALUE[,KEY=VALUE]) run in turn")
    p.add_argument("--out", default=str(ROOT / "gpurun_out" / "k20_timeline.jsonl"))
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    from config_lines import reserve_streams
    streams = reserve_streams(torch, a.inflight)
    import shine_amd
    from shine_amd import datasets as D
    L = shine_amd._lib
    base = D.sift_like(1_000_000, seed=1)
    B, nb = 1024, 12
    q = D.sift_like(B * nb, seed=2)
    with shine_amd.GpuBuild(base, 16, 200, L.METRIC_L2, seed=1234) as gb:
        idx = gb.open()
    qd = torch.from_numpy(q).cuda()
    ids = torch.empty((nb, B, 10), dtype=torch.int32, device="cuda")
    dists = torch.empty((nb, B, 10), dtype=torch.float32, device="cuda")
    qs = torch.zeros((nb, B, L.QS_WORDS), dtype=torch.int32, device="cuda")
    torch.cuda.set_stream(streams[0])

    def step(i, rec=None):
        b = i % nb
        s = streams[i % len(streams)]
        if rec is not None:
            rec[0].record(s)
        idx.knn_device(qd[b * B:(b + 1) * B].data_ptr(), B, 10, a.ef, ids[b].data_ptr(), dists[b].data_ptr(),
                       qs[b].data_ptr(), stream=s.cuda_stream)
        if rec is not None:
            rec[1].record(s)

    lines = []
    for mode, env in [(m, e) for m in a.mode.split(",") for e in (a.envs.split(";") if a.envs else [""])]:
        idx.set_search_mode(L.MODE_FAST if mode == "fast" else L.MODE_EXACT)
        kv = [x.partition("=") for x in env.split(",") if x]
        for k_, _, v_ in kv:
            os.environ[k_] = v_
        for i in range(nb):
            step(i)
        torch.cuda.synchronize()
        for rep in range(a.reps):
            for i in range(a.warmup):
                step(i)
            torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
            host = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                step(a.warmup + i, evs[i])
                host.append((time.perf_counter() - t0) * 1e3)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) * 1e3
            first = evs[0][0]
            starts = [first.elapsed_time(s) for s, _ in evs]
            ends = [first.elapsed_time(e) for _, e in evs]
            span = max(ends)
            d = {"env": env, "rep": rep, "steps": a.steps, "warmup": a.warmup, "mode": mode, "wall_ms": el, "span_ms": span,
                 "qps_wall": a.steps * B / el * 1e3, "qps_span": a.steps * B / span * 1e3,
                 "host_enqueue_ms": host, "start_ms": starts, "end_ms": ends,
                 "last_end_minus_second_last": sorted(ends)[-1] - sorted(ends)[-2]}
            log(f"{mode} {env or 'default'} rep {rep}: wall {el:.3f} ms span {span:.3f} ms; host enqueue done at {host[-1]:.3f} "
                f"ms (first {host[0]:.3f}); starts {[round(x, 3) for x in starts[:6]]}..; ends "
                f"{[round(x, 3) for x in sorted(ends)[-5:]]}")
            lines.append(d)
        for k_, _, _ in kv:
            del os.environ[k_]
    idx.close()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "a") as f:
        for d in lines:
            f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
