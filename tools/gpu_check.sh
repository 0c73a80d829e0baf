set -o pipefail
O=gpurun_out/${1:-check}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u tools/lib_probe.py --runs fast:48,fast:128,exact:128,exact:64 --tag ${1:-check} > $O/probe.jsonl 2> $O/probe.log || { echo probe failed; tail -20 $O/probe.log; exit 1; }
cat $O/probe.jsonl
