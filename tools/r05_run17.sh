#!/bin/bash
# Round 5, run 17: the largest u32 table at a given residency (LDS / wavefronts per CU): cfg4 100M at 6 and 7 per CU
# (6,400 / 5,440 entries), cfg5 50M at 4 and 5 per CU (9,536 / 7,488 entries).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes fast --cmp-oracle 0 --steps 100 \
  --envs "SHINE_DEBUG_VISCAP=6400;SHINE_DEBUG_VISCAP=5440;SHINE_DEBUG_VISCAP=6144" \
  --out gpurun_out/scale_cfg4_viscap3.jsonl > gpurun_out/scale_cfg4_viscap3.log 2>&1 || exit 3
timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes fast --cmp-oracle 0 --steps 60 \
  --envs "SHINE_DEBUG_VISCAP=9536;SHINE_DEBUG_VISCAP=7488;SHINE_DEBUG_VISCAP=9216" \
  --out gpurun_out/scale_cfg5_viscap2.jsonl > gpurun_out/scale_cfg5_viscap2.log 2>&1 || exit 4
echo ok
