#!/bin/bash
# Round 5, GPU call 9: cfg 5 at full size (TTI-shaped 50M x 200, fp16 rows, IP, ef 250, Zipf 1.0) with the oracle
# sample on the GPU-built dump (exact mode on f32 rows of the same graph).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/scale_lines.py --which cfg5 --out gpurun_out/scale_cfg5_r05i.jsonl > gpurun_out/scale_cfg5_r05i.log 2>&1 || exit 1
