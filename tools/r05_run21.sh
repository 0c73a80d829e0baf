#!/bin/bash
# Round 5, run 21: the large-id test, then the bench as the driver runs it (K = 20, W = 5) and at its default (K = 200).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_ids.py -x -q --timeout 300 --timeout-method thread > gpurun_out/large_ids_r05g.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_k20_r05g.json 2> gpurun_out/bench_k20_r05g.log || exit 3
timeout -k 10 400 python -u bench.py > gpurun_out/bench_k200_r05g.json 2> gpurun_out/bench_k200_r05g.log || exit 4
echo ok
