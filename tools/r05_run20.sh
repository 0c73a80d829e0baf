#!/bin/bash
# Round 5, run 20: the fast table at load 0.45 of the mean query grown to its residency level; exact from the recent worst query;
# cfg4 100M and cfg5 50M, then the bench's K = 20 timeline (fast, exact) on the same build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHINE_DEBUG_SHAPE=1 timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes fast,exact --cmp-oracle 0 --steps 100 \
  --out gpurun_out/scale_cfg4_rule3.jsonl > gpurun_out/scale_cfg4_rule3.log 2>&1 || exit 3
SHINE_DEBUG_SHAPE=1 timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes fast,exact --cmp-oracle 0 --steps 60 \
  --out gpurun_out/scale_cfg5_rule3.jsonl > gpurun_out/scale_cfg5_rule3.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/k20_timeline.py --reps 3 --warmup 5 --mode fast,exact --out gpurun_out/k20_rule3.jsonl > gpurun_out/k20_rule3.log 2>&1 || exit 5
echo ok
