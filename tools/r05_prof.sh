#!/bin/bash
# Round-5 profiles (via gpurun): the default bench line under rocprofv3 kernel statistics and a kernel trace (span per
# launch), then the HBM-byte and SQ counter passes of the bench kernel and of the cfg5-shaped fp16 d=200 kernel
# (tools/pmc_probe_gpu.py), one pass per process under its own kill timer.  Usage: bash tools/r05_prof.sh <tag>
set -o pipefail
TAG=${1:-r05prof}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- \
  python3 -u $R/bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.json | cut -c1-300
T=$(find $O/prof -name "bench_kernel_trace.csv" | head -1)
python3 $R/tools/trace_span.py "$T" --skip 32 --count 200 --out $O/bench_fast_trace_span.json || exit 1
S=$(find $O/prof -name "bench_kernel_stats.csv" | head -1); cp "$S" $O/bench_kernel_stats.csv
rm -f "$T"
bash $R/tools/r04_pmc.sh $TAG/pmc sift1m_f32,cfg5_10m_f16 || exit 2
echo done
