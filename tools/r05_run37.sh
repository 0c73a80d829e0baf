#!/bin/bash
# Round 5, run 37: where the ACCT = 2 search kernel's time goes — the skew cell's +cache leg with the arena lookup as
# built (0), with every row read from its home copy and the lookup left to the accounting (1), and without the cbits
# test ahead of cslot (2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r37
for v in 0 1 2; do
  SHINE_DEBUG_CACHE_ROWS=$v SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 300 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels +cache --warm 8 --calls 8 --out gpurun_out/r37/cell_$v.jsonl > gpurun_out/r37/cell_$v.log 2>&1 || exit 2
done
echo ok
