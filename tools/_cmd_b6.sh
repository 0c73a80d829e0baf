mkdir -p gpurun_out/b6
export GPU_MAX_HW_QUEUES=8
bash tools/gpu_round.sh v11 20 || exit 1
for ef in 128 48; do
timeout -k 10 300 python -u tools/occupancy_probe.py --ef $ef --settings f32:4:0,f32:4:4096:940,u8:4:0,u8:4:4096:940,u8:6:4096:940,f32:6:0 --nbatches 24 --out gpurun_out/b6/occ_ef$ef.jsonl > gpurun_out/b6/occ_ef$ef.log 2>&1 || { tail -20 gpurun_out/b6/occ_ef$ef.log; exit 1; }
cat gpurun_out/b6/occ_ef$ef.jsonl
done
