#!/bin/bash
# Round 5, run 38: the skew cell's launch shapes (SHINE_DEBUG_SHAPE), baseline against +cache.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r38
SHINE_DEBUG_SHAPE=1 timeout -k 10 300 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/r38/cell.jsonl > gpurun_out/r38/cell.log 2>&1 || exit 2
echo ok
