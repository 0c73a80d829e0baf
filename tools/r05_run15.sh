#!/bin/bash
# Round 5, run 15: cfg4 at 100M, fast mode, the visited table's size against residency: the default (the worst query's
# u32 table), 5,120 entries (8 wavefronts per CU by LDS; queries past 4,480 visits spill to the L2 hash set), the
# mean-sized 4,096 (10 per CU).  The random-gather probe (profiles/r05/gather_probe*.jsonl) reads 12.8 G rows/s at 6
# wavefronts per CU and 15.0 G at 8 for 384-byte rows, 10 rows a step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes fast --cmp-oracle 0 --steps 100 \
  --envs ";SHINE_DEBUG_VISCAP=5120;SHINE_DEBUG_VISCAP=4096;SHINE_DEBUG_VISCAP=6144" \
  --out gpurun_out/scale_cfg4_viscap.jsonl > gpurun_out/scale_cfg4_viscap.log 2>&1 || exit 3
echo ok
