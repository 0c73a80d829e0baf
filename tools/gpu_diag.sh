#!/bin/bash
# Isolating run: one test selection per step, each step stops the script on failure (no GPU step after a fault).
set -o pipefail
O=gpurun_out/${1:-diag}; mkdir -p $O; shift
export TMPDIR=/tmp
i=0
for sel in "$@"; do
  i=$((i+1))
  echo "== step $i: $sel"
  env $sel > $O/step$i.log 2>&1
  rc=$?
  tail -25 $O/step$i.log
  if [ $rc -ne 0 ]; then echo "step $i failed rc=$rc"; exit 1; fi
done
