#!/bin/bash
# Round-3 counter evidence (via gpurun): SQ counter passes of one 1,024-query batch on the bench's index for the exact
# kernel (f32 rows) and the fast kernel (f32 and u8 rows), and the phase profiles.  Usage: bash tools/prof_r03.sh <tag>
set -o pipefail
TAG=${1:-prof}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BUILD_ONLY=1 timeout -k 10 300 python3 $R/tools/pmc_probe.py > $O/build.log 2>&1 || { echo build failed; exit 1; }
for CASE in exact:f32 fast:f32 fast:u8; do
  MODE=${CASE%%:*}; ROWS=${CASE##*:}; T=${MODE}_${ROWS}
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_INSTS_BRANCH TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES"; do
    i=$((i+1))
    ROWS=$ROWS MODE=$MODE timeout -s KILL 120 rocprofv3 --pmc $P -d $O/${T}_p$i -o run --output-format csv -- python3 $R/tools/pmc_probe.py > $O/${T}_p$i.log 2>&1 || { echo "pass $T $i failed"; tail -5 $O/${T}_p$i.log; exit 1; }
  done
  KT=float; [ $ROWS = u8 ] && KT="unsigned char"
  KN="search_fast_kernel<128, 0, $KT, 2, 2"; [ $MODE = exact ] && KN="search_kernel<128, 0, $KT, 0, 0"
  python3 $R/tools/pmc_summary.py $O/${T}_p*/run_counter_collection.csv --kernel "$KN" --out $O/sq_$T.json
  V=1; [ $MODE = exact ] && V=0
  SHINE_DEBUG_VIS16=$V ROWS=$ROWS MODE=$MODE timeout -k 10 120 python3 $R/tools/phase_profile.py > $O/phase_$T.log 2>&1 || { echo phase failed; tail -5 $O/phase_$T.log; exit 1; }
  cat $O/phase_$T.log
done
echo done
