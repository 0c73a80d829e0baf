#!/bin/bash
# Round 5, run 26: the cache engine with records carrying slot / device / cooling bit and a draw ring — the GPU cache
# tests, then the skew cell (alpha 1.0, ratio 5 %) with per-slot replay timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cache_tests_r05k.txt 2>&1 || exit 2
SHINE_DEBUG_CACHE_TIMING=2 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/skew_cell_r05k.jsonl > gpurun_out/skew_cell_r05k.log 2>&1 || exit 4
echo ok
