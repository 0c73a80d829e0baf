#!/bin/bash
# Round 5, run 33: the exact pass's u32 table at load 0.45 of the mean query, grown to its residency level, beyond L2
# (SHINE_EXACT_LOAD_RULE, default on) against off — cfg4 100M and cfg5 50M exact, with the shapes printed; then the
# large-id and parity GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHINE_DEBUG_SHAPE=1 timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --modes exact --cmp-oracle 0 --steps 60 \
  --out gpurun_out/scale_cfg4_exact_rule2.jsonl > gpurun_out/scale_cfg4_exact_rule2.log 2>&1 || exit 3
SHINE_DEBUG_SHAPE=1 timeout -k 10 900 python -u tools/scale_lines.py --which cfg5 --modes exact --cmp-oracle 0 --steps 30 \
  --out gpurun_out/scale_cfg5_exact_rule2.jsonl > gpurun_out/scale_cfg5_exact_rule2.log 2>&1 || exit 4
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_ids.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exact_rule2_tests.txt 2>&1 || exit 5
echo ok
