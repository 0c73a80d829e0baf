set -o pipefail
O=gpurun_out/hwq; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-host --ef-sweep '' --no-rows-compare --mode fast > $O/q4.json 2> $O/q4.log || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-host --ef-sweep '' --no-rows-compare --mode fast > $O/q8.json 2> $O/q8.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr4 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu --no-host --ef-sweep '' --no-rows-compare --mode fast > $O/tr4.json 2> $O/tr4.log || exit 1
python - <<'PY'
import json
for f in ("q4", "q8", "tr4"):
    d = json.loads(open(f"gpurun_out/hwq/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d.get("hw_queues"))
PY
