#!/bin/bash
# Round 5, GPU call 8: the compute-node façade (with shine_prepare), the skew cell with prefetching evictions, the bench
# at K = 200 (default) and K = 20.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/compute_node_run.py --out gpurun_out/compute_node_r05h.jsonl > gpurun_out/compute_node_r05h.log 2>&1 || exit 1
SHINE_DEBUG_CACHE_TIMING=2 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 24 --calls 8 --out gpurun_out/skew_cell_r05h.jsonl > gpurun_out/skew_cell_r05h.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/bench_r05h.json 2> gpurun_out/bench_r05h.err || exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_r05h_k20.json 2> gpurun_out/bench_r05h_k20.err || exit 4
