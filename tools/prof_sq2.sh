#!/bin/bash
# Counter passes of the fast kernel with two batches' worth of wavefronts in ONE dispatch (NQ=2048: 8 wavefronts per
# CU, the residency of two 1,024-query batches in flight), so per-dispatch counters show the shared-CU regime.
set -o pipefail
TAG=${1:-sq2}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp NQ=${NQ:-2048}
BUILD_ONLY=1 timeout -k 10 300 python3 $GRAFT_REPO_ROOT/tools/pmc_probe.py > $O/build.log 2>&1 || { echo build failed; exit 1; }
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pmc_probe.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O/p*/run_counter_collection.csv --kernel search_fast_kernel --out $O/summary.json
