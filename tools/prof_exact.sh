#!/bin/bash
# Exact-mode evidence: rocprofv3 kernel stats of the bench run in exact mode, SQ counter passes of
# search_kernel on one 1,024-query batch (MODE=exact), and the phase profile of the exact kernel.
# Usage (via gpurun): bash tools/prof_exact.sh <tag>
set -o pipefail
TAG=${1:-exact}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BUILD_ONLY=1 timeout -k 10 300 python3 $R/tools/pmc_probe.py > $O/build.log 2>&1 || { echo build failed; exit 1; }
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-host --mode exact --ef-sweep '' --no-rows-compare > $O/bench_exact.json 2> $O/bench_exact.log || { echo prof failed; tail -20 $O/bench_exact.log; exit 1; }
cat $O/bench_exact.json
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_INSTS_BRANCH TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_TOTAL_CACHE_ACCESSES TCP_TCP_TA_DATA_STALL_CYCLES"; do
  i=$((i+1))
  MODE=exact timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 $R/tools/pmc_probe.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O/p*/run_counter_collection.csv --kernel 'search_kernel<128, 0, float, 0, false' --out $O/sq_summary.json
SHINE_DEBUG_VIS16=0 MODE=exact timeout -k 10 120 python3 $R/tools/phase_profile.py > $O/phase.log 2>&1 || { echo phase failed; tail -5 $O/phase.log; exit 1; }
cat $O/phase.log
echo done
