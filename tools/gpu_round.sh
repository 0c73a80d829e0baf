#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes.
# bench.py sets 8 hardware queues for itself; under rocprofv3 HIP may start first, so those lines set it too.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [steps]
set -o pipefail
TAG=${1:-run}; STEPS=${2:-20}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 500 python -u bench.py --steps $STEPS --warmup 5 > $O/bench.json 2> $O/bench.log || { echo bench failed; tail -30 $O/bench.log; exit 1; }
cat $O/bench.json
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu --no-host --mode fast --ef-sweep '' > $O/bench_prof.json 2> $O/bench_prof.log || { echo prof failed; tail -20 $O/bench_prof.log; exit 1; }
GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-host --nbatches 4 --mode fast --ef-sweep '' > $O/pmc_fetch.json 2> $O/pmc_fetch.log || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-host --nbatches 4 --mode fast --ef-sweep '' > $O/pmc_write.json 2> $O/pmc_write.log || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
python tools/trace_span.py $O/prof/run_kernel_trace.csv --skip $((12 + 5)) --count $STEPS --out $O/trace_span.json
python tools/pmc.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv --kernel 'search_fast_kernel<128, 0, float, 2, 2' --out $O/pmc.json
echo done
