#!/bin/bash
# Round 5, GPU call 7: the -m gpu suite (u16 tables on ties, flat cache engine), the dynamic cache's skew cell, the
# compute-node façade end to end at 1M.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_r05g.log 2>&1 || exit 1
SHINE_DEBUG_CACHE_TIMING=2 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 24 --calls 8 --out gpurun_out/skew_cell_r05g.jsonl > gpurun_out/skew_cell_r05g.log 2>&1 || exit 2
timeout -k 10 600 python -u tools/compute_node_run.py --out gpurun_out/compute_node_r05g.jsonl > gpurun_out/compute_node_r05g.log 2>&1 || exit 3
