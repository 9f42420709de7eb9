#!/bin/bash
# matrix-core GPU tests (all MFMA kernels) + the rocSPARSE comparator
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 120 --timeout-method thread -k "mfma or rocsparse or c2_full" > gpurun_out/t_mfma.log 2>&1; tail -4 gpurun_out/t_mfma.log
