#!/bin/bash
# Exact-mode table sizing at the bench config (diagnostics, via gpurun): tools/lib_probe.py per env variant, alternated.
set -o pipefail
O=gpurun_out/exact_scan; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "48 2" "32 2" "24 2" "32 3"; do
    set -- $v
    SHINE_EXACT_TABLE_PER_EF=$1 SHINE_EXACT_TARGET_BATCHES=$2 timeout -k 10 300 python -u tools/lib_probe.py --runs exact:128,exact:64 --tag "per_ef=$1,batches=$2" >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe $v failed"; tail -20 $O/probe.log; exit 1; }
  done
done
cat $O/probe.jsonl
