#!/bin/bash
# Round 5, run 42: the ACCT = 2 kernels with one held-back log entry per lane and kind (flushed by the wave when a lane
# must log a second entry, and at the end of the query) — the GPU cache tests, the skew cell on 8 and on 2 slots.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r42
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/cache_tests.txt 2>&1 || { tail -30 $O/cache_tests.txt; exit 2; }
tail -1 $O/cache_tests.txt
SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 300 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out $O/cell8.jsonl > $O/cell8.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/skew_grid.py --slots 2 --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out $O/cell2.jsonl > $O/cell2.log 2>&1 || exit 4
echo ok
