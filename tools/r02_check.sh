#!/bin/bash
# GPU tests, then a cross-build A/B, a batches-in-flight check and the cfg5 skew grid.  Usage: bash tools/r02_check.sh <tag>
set -o pipefail
O=gpurun_out/${1:-check}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u tools/ab_lib.py --libs "_abl/libshine_r01.so,dm-hnsw-reference_amd/libshine_gpu.so" --ef 32,64,128 --reps 3 > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
grep -v "^\[bench" $O/ab.log | grep qps_median | cut -c1-110
for n in 2 3; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --nbatches 12 --inflight $n --no-cpu --no-host --mode fast --ef-sweep '' > $O/bench_inflight$n.json 2> $O/bench_inflight$n.log || { echo bench $n failed; tail -20 $O/bench_inflight$n.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_inflight$n.json').read().strip().splitlines()[-1]); print('inflight', $n, d['value'], d['roofline']['frac'])"
done
timeout -k 10 400 python -u tools/config_lines.py --which cfg5skew --n 1000000 --out $O/cfg5_skew.jsonl > $O/cfg5_skew.log 2>&1 || { echo skew failed; tail -20 $O/cfg5_skew.log; exit 1; }
grep -h hit_rate $O/cfg5_skew.jsonl | cut -c1-300
echo done
