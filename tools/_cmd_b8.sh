mkdir -p gpurun_out/b8
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python -u tools/host_leg_probe.py --out gpurun_out/b8/host.jsonl > gpurun_out/b8/host.log 2>&1 || { tail -20 gpurun_out/b8/host.log; exit 1; }
cat gpurun_out/b8/host.jsonl
