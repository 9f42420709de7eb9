set -e
mkdir -p gpurun_out/glds
echo '{"MFMA_GLDS": 4}' > gpurun_out/glds/g4.json
timeout -k 10 200 python3 -u scripts/shape_sweep.py c2 20:2:0 > gpurun_out/glds/c2_g2.log 2>&1
GS_CONFIG=$PWD/gpurun_out/glds/g4.json timeout -k 10 200 python3 -u scripts/shape_sweep.py c2 20:2:0 > gpurun_out/glds/c2_g4.log 2>&1
timeout -k 10 200 python3 -u scripts/shape_sweep.py attn 28:2:0 > gpurun_out/glds/attn_g2.log 2>&1
GS_CONFIG=$PWD/gpurun_out/glds/g4.json timeout -k 10 200 python3 -u scripts/shape_sweep.py attn 28:2:0 > gpurun_out/glds/attn_g4.log 2>&1
grep -h -v amdgpu gpurun_out/glds/*.log
