#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_api_probe.py --out gpurun_out/host_api_probe_r05d.jsonl > gpurun_out/host_api_probe_r05d.log 2>&1 || exit 3
SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/skew_cell_r05d.jsonl > gpurun_out/skew_cell_r05d.log 2>&1 || exit 4
timeout -k 10 420 python -u tools/large_ids_probe.py 2>&1 | tee gpurun_out/large_ids_probe_r05d.log || exit 5
