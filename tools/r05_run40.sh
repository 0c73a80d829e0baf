#!/bin/bash
# Round 5, run 40: the dynamic cache's kernel cost against slot count and batch — the skew cell (alpha 1.0, 5 %) on
# 2 slots (their two cslot tables fit the Infinity Cache) and on 8 slots with 8,192-query calls (1,024 per slot).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r40
mkdir -p $O
timeout -k 10 400 python -u tools/skew_grid.py --slots 2 --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out $O/slots2.jsonl > $O/slots2.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/skew_grid.py --slots 8 --batch 8192 --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out $O/batch8192.jsonl > $O/batch8192.log 2>&1 || exit 3
echo ok
