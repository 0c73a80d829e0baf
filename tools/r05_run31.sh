#!/bin/bash
# Round 5, run 31: bulk staging / result copies for in-order query runs — the host-API tests, the host-API probe
# (12,288 and 10,000 queries per call) and the compute-node façade.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_cache.py tests/test_compute_node.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bulk_tests.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/host_api_probe.py --nq 12288 --chunks 1024 --reps 10 --out gpurun_out/host_api_bulk.jsonl > gpurun_out/host_api_bulk.log 2>&1 || exit 3
timeout -k 10 600 python -u tools/compute_node_run.py --out gpurun_out/compute_node_bulk.jsonl > gpurun_out/compute_node_bulk.log 2>&1 || exit 5
echo ok
