#!/bin/bash
# Round 5, run 12: the exact pass's learned table margin (SHINE_EXACT_LEARN_EIGHTHS) at K = 20 / warmup 5 (the driver's
# run) and K = 200: a batch whose worst query visits just over 4,096 / (9/8) nodes puts the next call on its stream on
# 8,192 entries, and that one slow launch sets a 20-step run's time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
E=";SHINE_EXACT_LEARN_EIGHTHS=8;SHINE_EXACT_LEARN_EIGHTHS=7;SHINE_EXACT_LEARN_EIGHTHS=6"
timeout -k 10 300 python -u tools/k20_timeline.py --reps 4 --warmup 5 --mode exact --envs "$E" --out gpurun_out/k20_exact_eighths.jsonl > gpurun_out/k20_exact_eighths.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/k20_timeline.py --reps 2 --warmup 20 --steps 200 --mode exact --envs "$E" --out gpurun_out/k200_exact_eighths.jsonl > gpurun_out/k200_exact_eighths.log 2>&1 || exit 3
echo ok
