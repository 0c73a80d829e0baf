#!/bin/bash
# Exact-mode table sizing at the bench config (diagnostics, via gpurun): tools/lib_probe.py per env variant, alternated.
# Variants: "learned-size eighths, target batches, learned minimum".
set -o pipefail
O=gpurun_out/exact_scan3; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "9 3 2048" "13 2 1024"; do
    set -- $v
    SHINE_EXACT_LEARN_EIGHTHS=$1 SHINE_EXACT_TARGET_BATCHES=$2 SHINE_EXACT_LEARN_MIN=$3 timeout -k 10 300 python -u tools/lib_probe.py --runs exact:32,exact:48,exact:64,exact:96,exact:128 --tag "eighths=$1,batches=$2,min=$3" >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe $v failed"; tail -20 $O/probe.log; exit 1; }
  done
done
cat $O/probe.jsonl
