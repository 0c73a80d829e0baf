#!/bin/bash
# Cost of the fallback passes' launches at the 20-step window (diagnostics, via gpurun): the bench's fast mode with the
# full pass chain against the main pass alone (SHINE_DEBUG_MAIN_ONLY=1, valid only while no query is handed on: the
# bench checks every query's status), alternated.
set -o pipefail
O=gpurun_out/passes_k20; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for mo in 0 1; do
    for rows in f32 u8; do
      SHINE_DEBUG_MAIN_ONLY=$mo timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --rows $rows --no-cpu --no-host --mode fast --ef-sweep '' --no-rows-compare > $O/b.json 2> $O/b_${mo}_$rows.log || { echo "bench $mo $rows failed"; tail -20 $O/b_${mo}_$rows.log; exit 1; }
      python3 -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'main_only':$mo,'rows':'$rows','value':d['value'],'avg_launch_ms':d['roofline']['avg_launch_ms']}))" | tee -a $O/summary.jsonl
    done
  done
done
