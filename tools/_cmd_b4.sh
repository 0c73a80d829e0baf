mkdir -p gpurun_out/b4
for cfg in "20 2" "20 4" "100 2" "100 4" "20 3"; do set -- $cfg
timeout -k 10 300 python -u bench.py --steps $1 --inflight $2 --nbatches 12 --mode fast --no-host --no-cpu --no-rows-compare > gpurun_out/b4/s$1_if$2.json 2> gpurun_out/b4/s$1_if$2.log || { tail -20 gpurun_out/b4/s$1_if$2.log; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/b4/s$1_if$2.json'))
print('steps $1 inflight $2', round(d['value']/1e6,3), [(x['ef'],round(x['value']/1e6,2)) for x in d['ef_sweep']])"
done
