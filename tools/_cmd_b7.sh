mkdir -p gpurun_out/b7
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python -u tools/host_leg_probe.py --out gpurun_out/b7/host.jsonl > gpurun_out/b7/host.log 2>&1 || { tail -20 gpurun_out/b7/host.log; exit 1; }
cat gpurun_out/b7/host.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/b7/tr -o run --output-format csv -- python3 tools/host_leg_probe.py --variants full:4 --steps 40 > gpurun_out/b7/tr.log 2>&1 || { tail -20 gpurun_out/b7/tr.log; exit 1; }
ls gpurun_out/b7/tr
