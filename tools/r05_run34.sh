#!/bin/bash
# Round 5, run 34: cfg5 50M exact with two-choice u16 entries allowed on the learned table (SHINE_EXACT_TWO_CHOICE=1:
# 16,384 entries in the 32 KiB that hold 8,192 u32 ones) against the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHINE_DEBUG_SHAPE=1 timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes exact --cmp-oracle 0 --steps 30 \
  --envs ";SHINE_EXACT_TWO_CHOICE=1" --out gpurun_out/scale_cfg5_exact_tc.jsonl > gpurun_out/scale_cfg5_exact_tc.log 2>&1 || exit 4
echo ok
