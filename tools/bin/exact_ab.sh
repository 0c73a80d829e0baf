# A/B of exact-pass tuning hooks on the bench (K = 20): each argument is a comma-separated KEY=VALUE set
set -o pipefail
O=gpurun_out/exact_ab2; mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i+1))
  ( IFS=','; for kv in $spec; do export "$kv"; done
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_$i.json 2> $O/bench_$i.log ) || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/bench_$i.json') if l.startswith('{')][0]; print('$spec', round(d['value']), d['modes']['exact'])"
done
