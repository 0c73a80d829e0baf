mkdir -p gpurun_out/b1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b1/tests.log 2>&1 || { tail -30 gpurun_out/b1/tests.log; exit 1; }
tail -2 gpurun_out/b1/tests.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u tools/ab_lib.py --libs _abl/libshine_head.so,dm-hnsw-reference_amd/libshine_gpu.so --ef 32,64,128 > gpurun_out/b1/ab.json 2> gpurun_out/b1/ab.log || { tail -20 gpurun_out/b1/ab.log; exit 1; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u tools/ab_lib.py --libs _abl/libshine_head.so,dm-hnsw-reference_amd/libshine_gpu.so --ef 64,128 --mode exact --steps 50 --reps 3 > gpurun_out/b1/ab_exact.json 2> gpurun_out/b1/ab_exact.log || { tail -20 gpurun_out/b1/ab_exact.log; exit 1; }
tail -4 gpurun_out/b1/ab_exact.log
tail -8 gpurun_out/b1/ab.log
timeout -k 10 300 python -u tools/occupancy_probe.py --settings f32:2:0,f32:2:4096,f32:3:0,f32:3:4096,u8:2:0,u8:3:0,u8:4:0,u8:3:4096,u8:4:4096,u8:2:4096 --out gpurun_out/b1/occ.jsonl > gpurun_out/b1/occ.log 2>&1 || { tail -20 gpurun_out/b1/occ.log; exit 1; }
cat gpurun_out/b1/occ.jsonl
