"""Span check for overlapped launches: the GPU span of bench.py's K timed launches from a rocprofv3 kernel trace.

With two batches in flight the launches overlap, so a launch's HIP-event time (which includes waiting for CUs the
other batch still holds) and rocprofv3's per-dispatch duration (first wave to last) differ; what both clocks must
agree on is the span of the K timed launches, which bench.py reports as roofline.span_ms_per_launch.

Usage: python tools/trace_span.py <run_kernel_trace.csv> --skip 15 --count 20 [--kernel substr] [--out f.json]
(skip = validation batches + warmup launches of the timed configuration, in dispatch order)
"""
import argparse
import csv
import json

import numpy as np

p = argparse.ArgumentParser()
p.add_argument("trace")
p.add_argument("--kernel", default="search_fast_kernel<128, 0, float, 2, 2,")
p.add_argument("--skip", type=int, default=15)
p.add_argument("--count", type=int, default=20)
p.add_argument("--out")
a = p.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
t = rows[a.skip:a.skip + a.count]
start = min(int(r["Start_Timestamp"]) for r in t)
end = max(int(r["End_Timestamp"]) for r in t)
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in t]
out = {"kernel": a.kernel, "launches": len(t), "span_ms_per_launch": (end - start) / 1e6 / len(t),
       "mean_dispatch_ms": float(np.mean(dur)), "queues": sorted({r["Queue_Id"] for r in t})}
print(json.dumps(out, indent=1))
if a.out:
    open(a.out, "w").write(json.dumps(out, indent=1) + "\n")
