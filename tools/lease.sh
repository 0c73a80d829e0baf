#!/bin/bash
# One GPU lease (via gpurun), as a list of named steps run in order.  Every step runs under its own kill timer, its
# output goes to gpurun_out/<tag>/<step>.*, and the first failing step ends the lease (no retries: a GPU fault or a
# timeout stops everything after it).  Replaces the per-call one-off scripts of rounds 2-5.
#
# Usage: bash tools/lease.sh <tag> <step>[=arg] ...
#   tests[=FILES]        pytest -m gpu (FILES: comma-separated test files; default the whole suite)
#   smoke                __graft_entry__.smoke()
#   bench[=K]            bench.py as the driver runs it (K steps, default 20, warmup 5)
#   bench_prof[=K]       bench.py under rocprofv3 --kernel-trace --stats (default K = 200), trace span per launch
#   pmc[=WORKLOADS]      FETCH_SIZE / WRITE_SIZE and SQ counter passes (tools/r04_pmc.sh; sift1m_f32,sift1m_u8,cfg5_10m_f16)
#   scale=WHICH[:ARGS]   tools/scale_lines.py --which WHICH (cfg3 / cfg4 / cfg5 / cmp ...), ARGS: extra flags, "+" for " "
#   skew[=SLOTS]         one skew-grid cell (alpha 1.0, 5 % cache), baseline and +cache, on SLOTS slots (default 8)
#   host_api             tools/host_api_probe.py
#   compute_node         tools/compute_node_run.py (the compute-node facade on big-ann files)
#   k20                  tools/k20_timeline.py (fast and exact)
#   phase=WORKLOAD       tools/phase_profile.py (bench) or tools/phase_profile_cfg5.py (cfg5[:N records])
# Environment: every KEY=VALUE in LEASE_ENV (';'-separated) is exported for the whole lease (library hooks).
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
IFS=';' read -ra ENVS <<< "${LEASE_ENV:-}"
for kv in "${ENVS[@]}"; do [ -n "$kv" ] && export "$kv"; done

run() {  # run <name> <seconds> <command...>: stdout to <name>.out, stderr to <name>.log
  local name=$1 secs=$2; shift 2
  echo "[lease $(date +%H:%M:%S)] $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.log"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $name failed with $rc"; tail -25 "$O/$name.log"; tail -5 "$O/$name.out"; exit 1
  fi
  tail -2 "$O/$name.out" | cut -c1-400
}

for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  case $name in
    tests)
      files=${arg//,/ }
      run tests 900 python -u -m pytest ${files:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke)
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run bench_k${arg:-20} 500 python -u bench.py --steps ${arg:-20} --warmup 5 ;;
    bench_prof)
      K=${arg:-200}
      ( cd /tmp && export TMPDIR=/tmp && run bench_prof 500 rocprofv3 --kernel-trace --stats -d "$O/prof" -o bench \
          --output-format csv -- python3 -u "$R/bench.py" --steps $K ) || exit 1
      T=$(find "$O/prof" -name "bench_kernel_trace.csv" | head -1)
      python3 tools/trace_span.py "$T" --skip 32 --count $K --out "$O/bench_fast_trace_span.json" || exit 1
      S=$(find "$O/prof" -name "bench_kernel_stats.csv" | head -1); cp "$S" "$O/bench_kernel_stats.csv"
      rm -rf "$O/prof" ;;
    pmc)
      bash tools/r04_pmc.sh "$TAG/pmc" "${arg:-sift1m_f32}" || exit 1 ;;
    scale)
      which=${arg%%:*}; extra=""; [ "$which" != "$arg" ] && extra=${arg#*:}
      run scale_$which 1150 python -u tools/scale_lines.py --which "$which" ${extra//+/ } \
        --out "$O/scale_$which.jsonl" ;;
    skew)
      run skew${arg:-8} 600 python -u tools/skew_grid.py --slots ${arg:-8} --alphas 1.0 --ratios 5 \
        --labels baseline,+cache --warm 8 --calls 8 --out "$O/skew${arg:-8}.jsonl" ;;
    host_api)
      run host_api 400 python -u tools/host_api_probe.py --out "$O/host_api.jsonl" ;;
    compute_node)
      run compute_node 600 python -u tools/compute_node_run.py --out "$O/compute_node.jsonl" ;;
    k20)
      run k20 400 python -u tools/k20_timeline.py --reps 3 --warmup 5 --mode fast,exact --out "$O/k20.jsonl" ;;
    phase)
      # (the library prints the phase totals to stderr: phase*.log)
      if [ "${arg%%:*}" = cfg5 ]; then n=10000000; [ "$arg" != cfg5 ] && n=${arg#*:}
        run phase_cfg5_$n 600 python -u tools/phase_profile_cfg5.py --n $n
      else run phase 400 python -u tools/phase_profile.py; fi ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
done
echo "lease $TAG done"
