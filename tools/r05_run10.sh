#!/bin/bash
# Round 5, run 10: the K = 20 timeline of the bench loop (fast and exact), and the skew cell with the reworked cache
# engine (per-slot replay timing at SHINE_DEBUG_CACHE_TIMING=2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/k20_timeline.py --reps 5 --out gpurun_out/k20_timeline_fast.jsonl > gpurun_out/k20_fast.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/k20_timeline.py --reps 5 --mode exact --out gpurun_out/k20_timeline_exact.jsonl > gpurun_out/k20_exact.log 2>&1 || exit 3
SHINE_DEBUG_CACHE_TIMING=2 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/skew_cell_r05e.jsonl > gpurun_out/skew_cell_r05e.log 2>&1 || exit 4
echo ok
