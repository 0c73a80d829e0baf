#!/bin/bash
# Round 5, run 18: the large-id-space fast table rule (no-spill over the recent calls, grown to its residency level;
# one wavefront more where residency is scarce) on cfg4 100M and cfg5 50M, fast and exact, with the shapes printed.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHINE_DEBUG_SHAPE=1 timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes fast,exact --cmp-oracle 0 --steps 100 \
  --out gpurun_out/scale_cfg4_rule.jsonl > gpurun_out/scale_cfg4_rule.log 2>&1 || exit 3
SHINE_DEBUG_SHAPE=1 timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes fast --cmp-oracle 0 --steps 60 \
  --envs ";SHINE_DEBUG_VISCAP=9536" --out gpurun_out/scale_cfg5_rule.jsonl > gpurun_out/scale_cfg5_rule.log 2>&1 || exit 4
echo ok
