mkdir -p gpurun_out/b2
for ef in 128 64 32; do
timeout -k 10 300 python -u tools/occupancy_probe.py --ef $ef --settings f32:2:0,f32:3:0,f32:4:0,f32:6:0,u8:2:0,u8:3:0,u8:4:0,u8:6:0 --nbatches 12 --out gpurun_out/b2/occ_ef$ef.jsonl > gpurun_out/b2/occ_ef$ef.log 2>&1 || { tail -20 gpurun_out/b2/occ_ef$ef.log; exit 1; }
cat gpurun_out/b2/occ_ef$ef.jsonl
done
