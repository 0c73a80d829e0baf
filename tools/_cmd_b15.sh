mkdir -p gpurun_out/b15
run() { local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --mode fast --no-host --no-cpu --no-rows-compare --ef-sweep 48 > gpurun_out/b15/$name.json 2> gpurun_out/b15/$name.log || { tail -20 gpurun_out/b15/$name.log; return 1; }
  python -c "
import json;d=json.load(open('gpurun_out/b15/$name.json'))
print('$name', round(d['value']/1e6,3), [(x['ef'],round(x['value']/1e6,2)) for x in d['ef_sweep']])"
}
run base A=1 && run noglobal SHINE_DEBUG_NO_GLOBAL=1 && run light64 SHINE_DEBUG_LIGHT_MIN_GRID=64 && run both SHINE_DEBUG_NO_GLOBAL=1 SHINE_DEBUG_LIGHT_MIN_GRID=64 && run base2 A=1 && run both2 SHINE_DEBUG_NO_GLOBAL=1 SHINE_DEBUG_LIGHT_MIN_GRID=64
