#!/bin/bash
# Round 5, run 27: the full skew grid (6 alpha x 6 ratios x baseline / +cache / +adaptive-routing, 24 warm-up calls,
# 8 measured) with the round-5 cache engine, then the cfg3 line (DEEP-shaped 10M, IP, ef 256, batch 4096).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/skew_grid.py --warm 24 --calls 8 --out gpurun_out/skew_grid_10m_r05.jsonl > gpurun_out/skew_grid_r05.log 2>&1 || exit 2
timeout -k 10 600 python -u tools/scale_lines.py --which cfg3 --modes fast,exact --cmp-oracle 0 --steps 60 \
  --out gpurun_out/scale_cfg3_r05.jsonl > gpurun_out/scale_cfg3_r05.log 2>&1 || exit 3
echo ok
