#!/bin/bash
# SQ / TA / TCP counter passes of the fast search kernel (one 1,024-query batch, tools/pmc_probe.py).
# Usage (via gpurun): bash tools/prof_sq.sh <tag>
set -o pipefail
TAG=${1:-sq}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BUILD_ONLY=1 timeout -k 10 300 python3 $GRAFT_REPO_ROOT/tools/pmc_probe.py > $O/build.log 2>&1 || { echo build failed; exit 1; }
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_INSTS_BRANCH TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pmc_probe.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O/p*/run_counter_collection.csv --kernel search_fast_kernel --out $O/sq_summary.json
