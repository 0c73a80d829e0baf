#!/bin/bash
# Round-4 counter passes (via gpurun): per workload, HBM bytes (FETCH_SIZE and WRITE_SIZE, one pass each) and two SQ
# passes (wave-cycle / wait mix; instruction mix, LDS conflicts, L2 latency) of the search kernel, on GPU-built
# indexes (tools/pmc_probe_gpu.py).  One pass per process, each under its own kill timer; the first failure ends it.
# Usage: bash tools/r04_pmc.sh <tag> [workloads: sift1m_f32,sift1m_u8,cfg5_10m_f16]
set -o pipefail
TAG=${1:-pmc}; WHICH=${2:-sift1m_f32,sift1m_u8,cfg5_10m_f16}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES"
for W in ${WHICH//,/ }; do
  case $W in
    sift1m_f32) export WORKLOAD=sift1m ROWS=f32; K="search_fast_kernel<128, 0, float, 2,"; T=150 ;;
    sift1m_u8) export WORKLOAD=sift1m ROWS=u8; K="search_fast_kernel<128, 0, unsigned char, 2,"; T=150 ;;
    cfg5_10m_f16) export WORKLOAD=cfg5_10m ROWS=f16; K="search_fast_kernel<200, 1, __half, 4,"; T=300 ;;
    cfg5_50m_f16) export WORKLOAD=cfg5_10m N=50000000 ROWS=f16 REPS=4; K="search_fast_kernel<200, 1, __half, 4, 2, 0, 3,"; T=420 ;;
    *) echo "unknown workload $W"; exit 1 ;;
  esac
  i=0; mkdir -p $O/$W
  for P in "FETCH_SIZE" "WRITE_SIZE" "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL $T rocprofv3 --pmc $P -d $O/$W/p$i -o run --output-format csv -- python3 $R/tools/pmc_probe_gpu.py \
      > $O/$W/p$i.log 2>&1 || { echo "$W pass $i failed"; tail -5 $O/$W/p$i.log; exit 1; }
    tail -1 $O/$W/p$i.log
  done
  python3 $R/tools/pmc.py $O/$W/p1/run_counter_collection.csv $O/$W/p2/run_counter_collection.csv --kernel "$K" \
    --out $O/${W}_pmc.json > /dev/null || { echo "$W pmc summary failed"; exit 1; }
  python3 $R/tools/pmc_summary.py $O/$W/p3/run_counter_collection.csv $O/$W/p4/run_counter_collection.csv --kernel "$K" \
    --out $O/${W}_sq.json > /dev/null || { echo "$W sq summary failed"; exit 1; }
  rm -rf $O/$W/p1 $O/$W/p2 $O/$W/p3 $O/$W/p4  # every dispatch of the build too: too large to bring back
  echo "$W done"
done
echo done
