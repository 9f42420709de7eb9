set -e
mkdir -p gpurun_out/krot
echo '{"MFMA_KROT": 1}' > gpurun_out/krot/cfg.json
timeout -k 10 240 python3 -u scripts/shape_sweep.py c2 20:2:0:0 20:2:0:1 20:2:0:0 20:2:0:1 > gpurun_out/krot/c2.log 2>&1
timeout -k 10 240 python3 -u scripts/shape_sweep.py attn 28:2:0:0 28:2:0:1 > gpurun_out/krot/attn.log 2>&1
timeout -k 10 300 python3 -u scripts/shape_sweep.py fc2 28:2:0:0 28:2:0:1 > gpurun_out/krot/fc2.log 2>&1
timeout -k 10 200 python3 -u scripts/time_nm.py 28672 7168 128 2000 > gpurun_out/krot/nm0.log 2>&1
GS_CONFIG=gpurun_out/krot/cfg.json timeout -k 10 200 python3 -u scripts/time_nm.py 28672 7168 128 2000 > gpurun_out/krot/nm1.log 2>&1
cat gpurun_out/krot/c2.log gpurun_out/krot/attn.log gpurun_out/krot/fc2.log | grep -v amdgpu.ids
echo "nm krot0: $(tail -1 gpurun_out/krot/nm0.log)"; echo "nm krot1: $(tail -1 gpurun_out/krot/nm1.log)"
GS_CONFIG=$PWD/gpurun_out/krot/cfg.json timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_nm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/krot/tests.log 2>&1
tail -2 gpurun_out/krot/tests.log
