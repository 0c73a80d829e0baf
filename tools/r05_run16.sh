#!/bin/bash
# Round 5, run 16: fast-mode visited table size at the large id spaces, with the L2 hash set as the spill target:
# cfg4 100M (6,144 entries ran at 4.80 M QPS against 4.2 M default in run 15) and cfg5 50M.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes fast --cmp-oracle 0 --steps 100 \
  --envs "SHINE_DEBUG_VISCAP=6144;SHINE_DEBUG_VISCAP=7168;SHINE_DEBUG_VISCAP=8192;" \
  --out gpurun_out/scale_cfg4_viscap2.jsonl > gpurun_out/scale_cfg4_viscap2.log 2>&1 || exit 3
timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes fast --cmp-oracle 0 --steps 60 \
  --envs ";SHINE_DEBUG_VISCAP=8192;SHINE_DEBUG_VISCAP=9216;SHINE_DEBUG_VISCAP=10240;SHINE_DEBUG_VISCAP=12288" \
  --out gpurun_out/scale_cfg5_viscap.jsonl > gpurun_out/scale_cfg5_viscap.log 2>&1 || exit 4
echo ok
