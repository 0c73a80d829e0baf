#!/bin/bash
# Round 5, run 41: SQ counters of the skew cell's search kernels (alpha 1.0, 5 %, 2 slots), ACCT = 1 (baseline) against
# ACCT = 2 (+cache), one counter pass per run, search kernels only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r41
mkdir -p $O
i=0
for P in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
         "SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $P --kernel-include-regex search_fast -d $O/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/skew_grid.py --slots 2 --alphas 1.0 --ratios 5 --labels baseline,+cache --warm 8 --calls 8 --out $O/cell$i.jsonl > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
du -sh $O
echo ok
