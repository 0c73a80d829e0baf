mkdir -p gpurun_out/b9
MODE=exact EF=128 SHINE_DEBUG_VIS16=0 timeout -k 10 300 python -u tools/phase_profile.py > gpurun_out/b9/exact.log 2>&1 || { tail -20 gpurun_out/b9/exact.log; exit 1; }
MODE=fast EF=128 timeout -k 10 200 python -u tools/phase_profile.py > gpurun_out/b9/fast.log 2>&1 || { tail -20 gpurun_out/b9/fast.log; exit 1; }
tail -6 gpurun_out/b9/exact.log gpurun_out/b9/fast.log
