# A/B of the dynamic cache's replay (SHINE_CACHE_ASYNC 0 / 1) in one skew cell, on 2 and 8 slots
set -o pipefail
O=gpurun_out/skew_ab; mkdir -p $O
for slots in 2 8; do for async in 0 1 0 1; do
  SHINE_CACHE_ASYNC=$async timeout -k 10 300 python -u tools/skew_grid.py --slots $slots --alphas 1.0 --ratios 5 \
    --labels +cache --warm 8 --calls 8 --out $O/skew${slots}_async${async}.jsonl > $O/log_${slots}_${async}.txt 2>&1 || exit 1
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/skew_ab/*.jsonl')):
    for l in open(f):
        d=json.loads(l); print(f.split('/')[-1], round(d['host_api_qps_including_cache_updates']), round(d['kernel_ms_per_call'],3), round(d['wall_ms_per_call'],3), round(d['cache_hit_rate'],4))
PY
