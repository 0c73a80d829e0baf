mkdir -p gpurun_out/b13
timeout -k 10 420 python -u tools/config_lines.py --which cfg5,sharded --steps 20 --nbatches 8 --out gpurun_out/b13/lines_1m.jsonl > gpurun_out/b13/lines_1m.log 2>&1 || { tail -20 gpurun_out/b13/lines_1m.log; exit 1; }
timeout -k 10 660 python -u tools/config_lines.py --which cfg3 --n 10000000 --steps 20 --nbatches 8 --out gpurun_out/b13/lines_cfg3_10m.jsonl > gpurun_out/b13/lines_cfg3.log 2>&1 || { tail -20 gpurun_out/b13/lines_cfg3.log; exit 1; }
python -c "
import json
for f in ['gpurun_out/b13/lines_1m.jsonl','gpurun_out/b13/lines_cfg3_10m.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['workload'], d['search_mode'], round(d['value']/1e6,3), d.get('recall_at_10'), d.get('roofline',{}).get('frac'))"
