mkdir -p gpurun_out/b14
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b14/tests.log 2>&1 || { tail -30 gpurun_out/b14/tests.log; exit 1; }
tail -2 gpurun_out/b14/tests.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u tools/ab_lib.py --libs _abl/libshine_prefilter.so,dm-hnsw-reference_amd/libshine_gpu.so --ef 64,128 --mode exact --steps 50 --reps 3 --inflight 4 --nbatches 12 > gpurun_out/b14/ab_exact.json 2> gpurun_out/b14/ab_exact.log || { tail -20 gpurun_out/b14/ab_exact.log; exit 1; }
grep qps_median gpurun_out/b14/ab_exact.log
