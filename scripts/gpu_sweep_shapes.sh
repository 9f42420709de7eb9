set -e
mkdir -p gpurun_out/sweep
timeout -k 10 240 python3 -u scripts/shape_sweep.py c2 ${C2V:-20:2:0 40:2:2 40:2:1 32:2:0 20:2:0} > gpurun_out/sweep/c2.log 2>&1
timeout -k 10 240 python3 -u scripts/shape_sweep.py attn ${ATTNV:-20:2:0 28:2:0 32:2:0 20:2:0} > gpurun_out/sweep/attn.log 2>&1
timeout -k 10 300 python3 -u scripts/shape_sweep.py fc1 ${FC1V:-20:2:0 28:2:0 56:2:0 64:2:0} > gpurun_out/sweep/fc1.log 2>&1
timeout -k 10 300 python3 -u scripts/shape_sweep.py fc2 ${FC2V:-20:2:0 28:2:0 28:2:2 32:2:2} > gpurun_out/sweep/fc2.log 2>&1
cat gpurun_out/sweep/*.log
