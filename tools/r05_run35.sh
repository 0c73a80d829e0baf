#!/bin/bash
# Round 5, run 35: the ACCT = 2 kernels with the cache lookups taken where the row is requested and the log stores
# deferred by one expansion — the GPU cache tests, then the skew cell (alpha 1.0, ratio 5 %) with per-slot timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cache_tests_r05l.txt 2>&1 || { tail -30 gpurun_out/cache_tests_r05l.txt; exit 2; }
tail -1 gpurun_out/cache_tests_r05l.txt
SHINE_DEBUG_CACHE_TIMING=2 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/skew_cell_r05l.jsonl > gpurun_out/skew_cell_r05l.log 2>&1 || exit 4
echo ok
