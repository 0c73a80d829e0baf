#!/bin/bash
# Round 5, run 11: exact mode after fast mode on one handle (bench.py's order) against exact alone, warmup 5 as in the
# driver's run, with the main pass's shapes printed (SHINE_DEBUG_SHAPE).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHINE_DEBUG_SHAPE=1 timeout -k 10 300 python -u tools/k20_timeline.py --reps 4 --warmup 5 --mode fast,exact --out gpurun_out/k20_timeline_fast_exact.jsonl > gpurun_out/k20_fast_exact.log 2>&1 || exit 2
SHINE_DEBUG_SHAPE=1 timeout -k 10 300 python -u tools/k20_timeline.py --reps 4 --warmup 5 --mode exact --out gpurun_out/k20_timeline_exact_only.jsonl > gpurun_out/k20_exact_only.log 2>&1 || exit 3
echo ok
