#!/bin/bash
# Round 5, GPU call 6: the low-ef shapes (u32 vs u16 tables), the dynamic cache's replay parts, then cfg 4 at full
# size (100M) with the hash-table spill against the id-space bitmap, and the oracle sample on the GPU-built dump.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ef_floor.py --efs 16,24,32,48,64 --envs ";SHINE_DEBUG_VIS16=1" --out gpurun_out/ef_floor_r05f.jsonl > gpurun_out/ef_floor_r05f.log 2>&1 || exit 1
SHINE_DEBUG_CACHE_TIMING=2 timeout -k 10 420 python -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels +cache --warm 24 --calls 4 --out gpurun_out/skew_cell_r05f.jsonl > gpurun_out/skew_cell_r05f.log 2>&1 || exit 2
timeout -k 10 840 python -u tools/scale_lines.py --which cfg4 --envs ";SHINE_SPILL_HASH=0" --out gpurun_out/scale_cfg4_r05f.jsonl > gpurun_out/scale_cfg4_r05f.log 2>&1 || exit 3
