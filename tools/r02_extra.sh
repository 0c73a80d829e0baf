#!/bin/bash
# Round-2 measurement lines beyond the bench (via gpurun): cfg5 skew grid, the sharded bench leg, a phase profile
# of the fast kernel and a batches-in-flight scan.  Usage: bash tools/r02_extra.sh <tag>
set -o pipefail
O=gpurun_out/${1:-extra}; mkdir -p $O
timeout -k 10 400 python -u tools/config_lines.py --which cfg5skew --n 1000000 --out $O/cfg5_skew.jsonl > $O/cfg5_skew.log 2>&1 || { echo skew failed; tail -20 $O/cfg5_skew.log; exit 1; }
grep -h hit_rate $O/cfg5_skew.jsonl | cut -c1-260
timeout -k 10 400 python -u bench.py --placement sharded --gpus 1 --slots 8 --n 1000000 --steps 20 --warmup 5 --cache-frac 0.05 > $O/sharded.json 2> $O/sharded.log || { echo sharded failed; tail -20 $O/sharded.log; exit 1; }
cut -c1-600 $O/sharded.json
SHINE_PHASE_PROFILE=1 timeout -k 10 200 python -u tools/phase_profile.py > $O/phase.log 2>&1 || { echo phase failed; tail -20 $O/phase.log; exit 1; }
tail -6 $O/phase.log
timeout -k 10 300 python -u tools/ab_lib.py --inflight 3 --libs "dm-hnsw-reference_amd/libshine_gpu.so,dm-hnsw-reference_amd/libshine_gpu.so@SHINE_DEBUG_VISCAP=4096" --ef 64,128 --reps 3 > $O/ab_inflight3.log 2>&1 || { echo ab3 failed; tail -20 $O/ab_inflight3.log; exit 1; }
grep -v "^\[bench" $O/ab_inflight3.log | grep qps_median | cut -c1-120
echo done
