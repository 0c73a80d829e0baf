#!/bin/bash
# Round 5, run 24: the compute-node façade with its results written straight into a preallocated array (10,000
# queries, --store-index --builder gpu, then --load-index), and its GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "compute_node" --timeout 250 --timeout-method thread > gpurun_out/cn_tests_r05j.txt 2>&1 || exit 2
timeout -k 10 600 python -u tools/compute_node_run.py --out gpurun_out/compute_node_flat.jsonl > gpurun_out/compute_node_flat.log 2>&1 || exit 5
echo ok
