#!/bin/bash
# Exact-mode table sizing at the bench config (diagnostics, via gpurun): tools/lib_probe.py per env variant, alternated.
# Variants: "learned-size eighths, target batches".
set -o pipefail
O=gpurun_out/exact_scan2; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "9 3" "10 3" "13 3" "9 2" "13 2"; do
    set -- $v
    SHINE_EXACT_LEARN_EIGHTHS=$1 SHINE_EXACT_TARGET_BATCHES=$2 timeout -k 10 300 python -u tools/lib_probe.py --runs exact:32,exact:64,exact:128,exact:256 --tag "eighths=$1,batches=$2" >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe $v failed"; tail -20 $O/probe.log; exit 1; }
  done
done
cat $O/probe.jsonl
