mkdir -p gpurun_out/b3
for q in 8 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/occupancy_probe.py --ef 128 --settings f32:4:0,f32:6:0,f32:8:0,u8:4:0,u8:8:0 --nbatches 24 --out gpurun_out/b3/occ_q$q.jsonl > gpurun_out/b3/occ_q$q.log 2>&1 || { tail -20 gpurun_out/b3/occ_q$q.log; exit 1; }
cat gpurun_out/b3/occ_q$q.jsonl
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/occupancy_probe.py --ef 48 --settings f32:2:0,f32:4:0,f32:8:0,u8:4:0,u8:8:0 --nbatches 24 --out gpurun_out/b3/occ_ef48.jsonl > gpurun_out/b3/occ_ef48.log 2>&1 || { tail -20 gpurun_out/b3/occ_ef48.log; exit 1; }
cat gpurun_out/b3/occ_ef48.jsonl
