#!/bin/bash
# rocprofv3 kernel stats and the timed window's trace span of the bench in exact mode (via gpurun).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-exact_stats}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-host --mode exact --ef-sweep '' --no-rows-compare > $O/bench_exact.json 2> $O/bench_exact.log || { echo prof failed; tail -20 $O/bench_exact.log; exit 1; }
python3 $R/tools/trace_span.py $O/prof/run_kernel_trace.csv --kernel 'search_kernel<128, 0, float, 0, 0' --skip 17 --count 20 --out $O/trace_span.json
grep search_ $O/prof/run_kernel_stats.csv | cut -c1-160
