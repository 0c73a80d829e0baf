#!/bin/bash
# GPU A/B pass (via gpurun): the GPU test suite on the in-tree build, then tools/lib_probe.py once per library per
# repetition, libraries alternated (one process per build).  Usage: LIBS="_abl/a.so _abl/b.so" bash tools/ab.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
RUNS=${RUNS:-fast:128,fast:48,exact:128,fast:128:u8,fast:48:u8}
for rep in 1 2; do
  for L in $LIBS; do
    SHINE_GPU_LIB=$L timeout -k 10 300 python -u tools/lib_probe.py --runs $RUNS --tag $L >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe $L failed"; tail -20 $O/probe.log; exit 1; }
  done
done
[ -f $O/probe.jsonl ] && cat $O/probe.jsonl; true
