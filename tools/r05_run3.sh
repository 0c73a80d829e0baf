#!/bin/bash
# Round 5, GPU call 3: the 27-bit-id test alone with its phase timing (pytest -s), the rest of the -m gpu suite, the
# host-API probe, one skew-grid cell with the dynamic cache's timing split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_ids.py -x -v -s --timeout 380 --timeout-method thread 2>&1 | tee gpurun_out/gputest_r05c_large.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --deselect tests/test_gpu_large_ids.py::test_spill_to_hash_at_27_bit_ids > gpurun_out/gputest_r05c.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/host_api_probe.py --out gpurun_out/host_api_probe_r05c.jsonl > gpurun_out/host_api_probe_r05c.log 2>&1 || exit 3
SHINE_DEBUG_CACHE_TIMING=1 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out gpurun_out/skew_cell_r05c.jsonl > gpurun_out/skew_cell_r05c.log 2>&1 || exit 4
