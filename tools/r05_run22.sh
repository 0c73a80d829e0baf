#!/bin/bash
# Round 5, run 22: u32 visited tables probing a 4-slot group per read — the GPU tests, then cfg4 100M (fast, exact),
# then the bench at its default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r05h.txt 2>&1 || exit 2
timeout -k 10 600 python -u tools/scale_lines.py --which cfg4 --modes fast,exact --cmp-oracle 0 --steps 100 \
  --out gpurun_out/scale_cfg4_group.jsonl > gpurun_out/scale_cfg4_group.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_k200_group.json 2> gpurun_out/bench_k200_group.log || exit 4
echo ok
