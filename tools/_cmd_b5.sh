mkdir -p gpurun_out/b5
run() { local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --inflight 4 --nbatches 12 --mode fast --no-host --no-cpu --no-rows-compare --ef-sweep 48 > gpurun_out/b5/$name.json 2> gpurun_out/b5/$name.log || { tail -20 gpurun_out/b5/$name.log; return 1; }
  python -c "
import json;d=json.load(open('gpurun_out/b5/$name.json'))
print('$name', round(d['value']/1e6,3), [(x['ef'],round(x['value']/1e6,2)) for x in d['ef_sweep']])"
}
run q_default A=1 && run q8 GPU_MAX_HW_QUEUES=8 && run q16 GPU_MAX_HW_QUEUES=16 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b5/tr -o run --output-format csv -- python3 bench.py --steps 20 --inflight 4 --nbatches 12 --mode fast --no-host --no-cpu --no-rows-compare --ef-sweep '' > gpurun_out/b5/tr.json 2> gpurun_out/b5/tr.log && \
python tools/trace_span.py gpurun_out/b5/tr/run_kernel_trace.csv --skip 17 --count 20 --out gpurun_out/b5/tr_span.json && cat gpurun_out/b5/tr_span.json
