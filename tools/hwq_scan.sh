#!/bin/bash
# bench.py fast leg under the default hardware-queue count and under 8 (diagnostics), interleaved.
set -o pipefail
O=gpurun_out/${1:-hwq}; mkdir -p $O
for rep in 1 2; do for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --nbatches 12 --no-cpu --no-host --mode fast --ef-sweep '' > $O/q${q}_$rep.json 2> $O/q${q}_$rep.log || { echo q$q failed; tail -5 $O/q${q}_$rep.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/q${q}_$rep.json').read().strip().splitlines()[-1]); print('queues $q rep $rep', round(d['value']), round(d['roofline']['frac'],3))"
done; done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-host --mode fast --ef-sweep '' > $O/q${q}_s20.json 2> $O/q${q}_s20.log || { echo q$q failed; exit 1; }
  python -c "import json; d=json.loads(open('$O/q${q}_s20.json').read().strip().splitlines()[-1]); print('queues $q steps 20', round(d['value']), round(d['roofline']['frac'],3))"
done
