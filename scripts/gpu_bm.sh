#!/bin/bash
# full GPU suite + default bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; tail -4 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --n-sweep 8,16,64,128 > gpurun_out/bench_default.log 2>&1; tail -c 3000 gpurun_out/bench_default.log
