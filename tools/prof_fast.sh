#!/bin/bash
# Fast-mode evidence: rocprofv3 kernel stats of the bench run, SQ counter passes of search_fast_kernel on one
# 1,024-query batch at ef=128 for f32 and u8 rows, and the phase profile of both.
# Usage (via gpurun): bash tools/prof_fast.sh <tag>
set -o pipefail
TAG=${1:-fast}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BUILD_ONLY=1 timeout -k 10 300 python3 $R/tools/pmc_probe.py > $O/build.log 2>&1 || { echo build failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-host --mode fast --ef-sweep '' > $O/bench_fast.json 2> $O/bench_fast.log || { echo prof failed; tail -20 $O/bench_fast.log; exit 1; }
for ROWS in f32 u8; do
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_INSTS_BRANCH TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES"; do
    i=$((i+1))
    ROWS=$ROWS MODE=fast timeout -s KILL 120 rocprofv3 --pmc $P -d $O/${ROWS}_p$i -o run --output-format csv -- python3 $R/tools/pmc_probe.py > $O/${ROWS}_p$i.log 2>&1 || { echo "pass $ROWS $i failed"; tail -5 $O/${ROWS}_p$i.log; exit 1; }
  done
  KT=float; [ $ROWS = u8 ] && KT="unsigned char"
  python3 $R/tools/pmc_summary.py $O/${ROWS}_p*/run_counter_collection.csv --kernel "search_fast_kernel<128, 0, $KT, 2, 2" --out $O/sq_summary_$ROWS.json
  ROWS=$ROWS MODE=fast timeout -k 10 120 python3 $R/tools/phase_profile.py > $O/phase_$ROWS.log 2>&1 || { echo phase failed; tail -5 $O/phase_$ROWS.log; exit 1; }
  cat $O/phase_$ROWS.log
done
echo done
