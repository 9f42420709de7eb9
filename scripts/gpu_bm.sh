#!/bin/bash
# every BASELINE config on the GPU
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_configs.log 2>&1; tail -15 gpurun_out/t_configs.log
