#!/bin/bash
# Round 5, run 25: PC sampling (rocprofv3 host-trap, beta) of the cfg5-shaped fast kernel (fp16 rows, d = 200, IP,
# ef = 250) on a 2M-record GPU-built index: which instructions the waves sit on.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pcs
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 -d $R/gpurun_out/pcs -o pcs --output-format csv -- \
  python3 -u $R/tools/phase_profile_cfg5.py --n 2000000 > $R/gpurun_out/pcs/run.log 2>&1 || { tail -30 $R/gpurun_out/pcs/run.log; exit 2; }
ls -la $R/gpurun_out/pcs
find $R/gpurun_out/pcs -name "*.csv" | head
echo ok
