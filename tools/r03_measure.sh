#!/bin/bash
# One GPU-box pass for round 3: the new config tests, the default bench line, and the per-mode probe of the bench
# workload.  Each step under its own time limit; the first failure ends the script (no GPU step after a fault).
# Usage (via gpurun): bash tools/r03_measure.sh <tag>
set -o pipefail
O=gpurun_out/${1:-m1}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "eight_slots_cached or dynamic_cache_exact" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -12 $O/bench.log
timeout -k 10 200 python -u tools/lib_probe.py --runs fast:48,fast:128,exact:128,exact:64,fast:128:u8,fast:48:u8 --tag r03 > $O/probe.jsonl 2> $O/probe.log || { echo "probe failed"; tail -30 $O/probe.log; exit 1; }
cat $O/probe.jsonl
# table sizing with in-place spill: smaller tables, sized for 16 waves per CU
SHINE_FAST_TARGET_BATCHES=4 SHINE_FAST_TABLE_PER_EF=24 timeout -k 10 200 python -u tools/lib_probe.py --runs fast:128,fast:128:u8,fast:48:u8 --tag small_tables >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe 2 failed"; tail -30 $O/probe.log; exit 1; }
# registers capped at 128 per lane (4 waves per SIMD)
if [ -f _abl/lib_w4.so ]; then
  SHINE_GPU_LIB=_abl/lib_w4.so timeout -k 10 200 python -u tools/lib_probe.py --runs fast:128,fast:128:u8,exact:128 --tag w4 >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe 3 failed"; tail -30 $O/probe.log; exit 1; }
  SHINE_GPU_LIB=_abl/lib_w4.so SHINE_FAST_TARGET_BATCHES=4 SHINE_FAST_TABLE_PER_EF=24 timeout -k 10 200 python -u tools/lib_probe.py --runs fast:128,fast:128:u8,fast:48:u8 --tag w4_small_tables >> $O/probe.jsonl 2>> $O/probe.log || { echo "probe 4 failed"; tail -30 $O/probe.log; exit 1; }
fi
cat $O/probe.jsonl
