#!/bin/bash
# Round 5: the final tree's GPU suite, smoke() and the bench as the driver runs it (K = 20, W = 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05check
O=gpurun_out/r05check
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 2; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.log || { tail -20 $O/bench_k20.log; exit 3; }
tail -1 $O/bench_k20.json | cut -c1-160
echo ok
