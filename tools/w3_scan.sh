#!/bin/bash
# f32 fast kernel at three waves per SIMD (a build with -DSHINE_FAST_MIN_WAVES=3) against the default build
# (diagnostics, via gpurun).  Variants: "library, fast target batches".
set -o pipefail
O=gpurun_out/w3_scan; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "dm-hnsw-reference_amd/libshine_gpu.so 2" "dm-hnsw-reference_amd/libshine_gpu.so 3" "w3/lib_w3.so 3" "w3/lib_w3.so 2"; do
    set -- $v
    SHINE_GPU_LIB=$1 SHINE_FAST_TARGET_BATCHES=$2 timeout -k 10 300 python -u tools/lib_probe.py --runs fast:128,fast:48 --tag "$1,batches=$2" >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe $v failed"; tail -20 $O/probe.log; exit 1; }
  done
done
cat $O/probe.jsonl
