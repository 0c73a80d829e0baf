#!/bin/bash
# Round 5, run 28: touch-ahead (SHINE_TOUCH_AHEAD=1: the rows of the candidate after next touched into L2) against
# off — the fast GPU tests with it on, then cfg5 50M, cfg4 100M and the bench's K = 20 / 200 loops.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHINE_TOUCH_AHEAD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/touch_tests.txt 2>&1 || exit 2
timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes fast --cmp-oracle 0 --steps 60 \
  --envs ";SHINE_TOUCH_AHEAD=1" --out gpurun_out/scale_cfg5_touch.jsonl > gpurun_out/scale_cfg5_touch.log 2>&1 || exit 3
timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes fast --cmp-oracle 0 --steps 100 \
  --envs ";SHINE_TOUCH_AHEAD=1" --out gpurun_out/scale_cfg4_touch.jsonl > gpurun_out/scale_cfg4_touch.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/k20_timeline.py --reps 3 --warmup 5 --mode fast --envs ";SHINE_TOUCH_AHEAD=1" --out gpurun_out/k20_touch.jsonl > gpurun_out/k20_touch.log 2>&1 || exit 5
echo ok
