#!/bin/bash
# Round-5 final evidence (via gpurun) on the round's last build: the GPU test suite and smoke(), the bench as the
# driver runs it (K = 20, W = 5), then the default bench line under rocprofv3 kernel statistics and a kernel trace
# (span per launch) and the HBM-byte / SQ counter passes of the bench kernel (tools/r04_pmc.sh).
# Usage: bash tools/r05_final.sh <tag>
set -o pipefail
TAG=${1:-r05final}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 2; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.log || { tail -20 $O/bench_k20.log; exit 3; }
tail -1 $O/bench_k20.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- \
  python3 -u $R/bench.py > $O/bench_k200.json 2> $O/bench_k200.log || { echo "bench failed"; tail -20 $O/bench_k200.log; exit 4; }
tail -1 $O/bench_k200.json | cut -c1-200
T=$(find $O/prof -name "bench_kernel_trace.csv" | head -1)
python3 $R/tools/trace_span.py "$T" --skip 32 --count 200 --out $O/bench_fast_trace_span.json || exit 5
S=$(find $O/prof -name "bench_kernel_stats.csv" | head -1); cp "$S" $O/bench_kernel_stats.csv
rm -rf $O/prof
bash $R/tools/r04_pmc.sh $TAG/pmc sift1m_f32 || exit 6
echo done
