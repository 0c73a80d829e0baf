#!/bin/bash
# One GPU-box pass (via gpurun): tests + A/B probe (tools/ab.sh), counter profile (tools/prof_r03.sh), then the
# default bench line.  Each step bounded; the first failure ends the script.  Usage: bash tools/r03_round.sh <tag>
set -o pipefail
T=${1:-r}; O=gpurun_out/$T; mkdir -p $O
bash tools/ab.sh $T || exit 1
if [ -z "$NO_PROF" ]; then bash tools/prof_r03.sh ${T}_prof > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }; tail -12 $O/prof.log; fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
  tail -8 $O/bench.log
fi
