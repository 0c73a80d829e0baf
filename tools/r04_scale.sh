#!/bin/bash
# Round-4 full-size config lines (via gpurun): cfg4 (DEEP-shaped 100M, L2, ef=128) and cfg5 (TTI-shaped 50M, IP, fp16
# rows, ef=250), each index built on the GPU in-run, under rocprofv3 kernel statistics.  Each step under its own time
# limit; the first failure ends the script.  Usage: bash tools/r04_scale.sh <tag> [workloads]
set -o pipefail
TAG=${1:-scale}; WHICH=${2:-cfg4,cfg5}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for W in ${WHICH//,/ }; do
  timeout -k 10 540 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- \
    python3 -u $R/tools/scale_lines.py --which $W --modes fast,exact --out $O/lines_$W.jsonl > $O/$W.log 2>&1 \
    || { echo "$W failed"; tail -20 $O/$W.log; exit 1; }
  grep -v '^{' $O/$W.log | grep -v '"workload"' | tail -4
  python3 - "$O" "$W" <<'EOF'
import json, sys
O, W = sys.argv[1], sys.argv[2]
for l in open(f"{O}/lines_{W}.jsonl"):
    d = json.loads(l)
    print(d["workload"], d["search_mode"], d["config"]["ef"], f"{d['value']:.0f} QPS", f"recall {d['recall_at_10']:.4f}",
          f"frac {d['roofline']['frac']:.3f}", f"build {d['build']['wall_s']:.1f}s")
EOF
done
echo done
