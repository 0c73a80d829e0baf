#!/bin/bash
# Round 5, run 36: kernel trace of the skew cell (alpha 1.0, ratio 5 %), baseline and +cache, for the search kernels'
# own durations (ACCT = 1 against ACCT = 2) and the cache apply kernels'.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof36
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof36/base -o run --output-format csv -- python3 -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels baseline --warm 8 --calls 8 --out gpurun_out/prof36/base.jsonl > gpurun_out/prof36/base.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof36/cache -o run --output-format csv -- python3 -u tools/skew_grid.py --alphas 1.0 --ratios 5 --labels +cache --warm 8 --calls 8 --out gpurun_out/prof36/cache.jsonl > gpurun_out/prof36/cache.log 2>&1 || exit 3
find gpurun_out/prof36 -name "*kernel_trace.csv" -delete; find gpurun_out/prof36 -name "*.db" -delete; du -sh gpurun_out/prof36; find gpurun_out/prof36 -name "*kernel_stats.csv"
echo ok
