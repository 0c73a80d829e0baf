#!/bin/bash
# Round-4 evidence (via gpurun): the GPU test suite, the default bench line under rocprofv3 kernel statistics and a
# kernel trace (span per launch), and the bench with the sharded leg at 10M records.  Each step under its own time
# limit; the first failure ends the script.  Usage: bash tools/r04_bench.sh <tag>
set -o pipefail
TAG=${1:-bench}; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- \
  python3 -u $R/bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.json | cut -c1-600
timeout -k 10 500 python3 -u $R/bench.py --gpus 1 --sharded-leg on --sharded-n 10000000 > $O/bench_sharded.json \
  2> $O/bench_sharded.log || { echo "sharded bench failed"; tail -20 $O/bench_sharded.log; exit 1; }
tail -1 $O/bench_sharded.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('sharded_leg', d.get('sharded')))[:1500])"
echo done
