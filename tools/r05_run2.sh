#!/bin/bash
# Round 5, GPU call 2: the -m gpu suite (hash spill, 27-bit ids, chunked host calls), the host-API probe, and one
# skew-grid cell with the dynamic cache's timing split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_r05b.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_api_probe.py --out gpurun_out/host_api_probe_r05b.jsonl > gpurun_out/host_api_probe_r05b.log 2>&1 || exit 2
SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/skew_cell_r05b.jsonl > gpurun_out/skew_cell_r05b.log 2>&1 || exit 3
