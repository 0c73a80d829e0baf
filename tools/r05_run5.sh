#!/bin/bash
# Round 5, GPU call 5: the -m gpu suite, the dynamic cache's skew cell pipelined and synchronous, the host-API probe,
# the low-ef floor.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_r05e.log 2>&1 || exit 1
SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 24 --calls 8 --out gpurun_out/skew_cell_r05e.jsonl > gpurun_out/skew_cell_r05e.log 2>&1 || exit 2
SHINE_CACHE_LAG=0 SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels +cache --warm 24 --calls 8 --out gpurun_out/skew_cell_r05e_sync.jsonl > gpurun_out/skew_cell_r05e_sync.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/host_api_probe.py --out gpurun_out/host_api_probe_r05e.jsonl > gpurun_out/host_api_probe_r05e.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/ef_floor.py --out gpurun_out/ef_floor_r05e.jsonl > gpurun_out/ef_floor_r05e.log 2>&1 || exit 5
