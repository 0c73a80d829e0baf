#!/bin/bash
# Batches in flight x visited-table size (diagnostics): bench.py fast mode, one process per setting.
set -o pipefail
O=gpurun_out/${1:-scan}; mkdir -p $O
run() {  # name ef inflight [VAR=VALUE]
  local name=$1 ef=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --nbatches 12 --inflight $n --ef $ef --no-cpu --no-host --mode fast --ef-sweep '' > $O/$name.json 2> $O/$name.log || { echo $name failed; tail -5 $O/$name.log; return 1; }
  python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']), d['recall_at_10'], round(d['roofline']['frac'],3))"
}
run ef64_if2 64 2 && run ef64_if3 64 3 && run ef64_if3_v2048 64 3 SHINE_DEBUG_VISCAP=2048 && run ef64_if2_v2048 64 2 SHINE_DEBUG_VISCAP=2048 && \
run ef128_if3_v4096 128 3 SHINE_DEBUG_VISCAP=4096 && run ef128_if4 128 4 && echo done
