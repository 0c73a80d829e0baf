#!/bin/bash
# Round 5, run 39: the host API with the first chunk of every host stream staged in parallel (default) against serial
# staging (SHINE_HOST_STAGE_PARALLEL=0): host_api_probe at 12,288 and 10,000 queries, the compute-node façade, then the
# GPU tests of the host path.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r39
mkdir -p $O
for p in 1 0 1 0; do
  SHINE_HOST_STAGE_PARALLEL=$p timeout -k 10 300 python -u tools/host_api_probe.py --nq 12288 --chunks 1024 --reps 20 --out $O/probe_p$p.jsonl >> $O/probe.log 2>&1 || exit 2
done
for p in 1 0; do
  SHINE_HOST_STAGE_PARALLEL=$p timeout -k 10 300 python -u tools/host_api_probe.py --nq 10000 --chunks 1024 --reps 20 --out $O/probe10k_p$p.jsonl >> $O/probe.log 2>&1 || exit 3
done
timeout -k 10 600 python -u tools/compute_node_run.py --out $O/compute_node.jsonl > $O/compute_node.log 2>&1 || exit 5
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 4; }
tail -1 $O/tests.txt
echo ok
