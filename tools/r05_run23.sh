#!/bin/bash
# Round 5, run 23: host-API chunks balanced over the host streams — the chunking test, the host-API probe at 10,000
# and 12,288 queries per call, and the compute-node façade (10,000 queries, --load-index after --store-index).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -x -q -k "chunks_in_flight" --timeout 200 --timeout-method thread > gpurun_out/chunk_test_r05i.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/host_api_probe.py --nq 10000 --chunks 1024 --reps 10 --out gpurun_out/host_api_balanced.jsonl > gpurun_out/host_api_balanced.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/host_api_probe.py --nq 12288 --chunks 1024 --reps 10 --out gpurun_out/host_api_balanced.jsonl >> gpurun_out/host_api_balanced.log 2>&1 || exit 4
timeout -k 10 600 python -u tools/compute_node_run.py --out gpurun_out/compute_node_balanced.jsonl > gpurun_out/compute_node_balanced.log 2>&1 || exit 5
echo ok
