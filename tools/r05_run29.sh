#!/bin/bash
# Round 5, run 29: cfg4 at 100M on the final build, fast and exact, with the CPU oracle's 64-query sample on the line's
# own dump (oracle_equals_exact_on_gpu_dump).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/scale_lines.py --which cfg4 --modes fast,exact --steps 100 \
  --out gpurun_out/scale_cfg4_final.jsonl > gpurun_out/scale_cfg4_final.log 2>&1 || exit 3
echo ok
