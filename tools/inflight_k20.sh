#!/bin/bash
# The driver's 20-step window against batches in flight (diagnostics, via gpurun): fast mode, f32 and u8 rows.
set -o pipefail
O=gpurun_out/inflight_k20; mkdir -p $O
export TMPDIR=/tmp
for n in 2 3 4 6 8; do
  for rows in f32 u8; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight $n --nbatches 24 --rows $rows --no-cpu --no-host --mode fast --ef-sweep '' --no-rows-compare > $O/b_${n}_$rows.json 2> $O/b_${n}_$rows.log || { echo "bench $n $rows failed"; tail -20 $O/b_${n}_$rows.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${n}_$rows.json'));print(json.dumps({'inflight':$n,'rows':'$rows','value':d['value'],'avg_launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" | tee -a $O/summary.jsonl
  done
done
