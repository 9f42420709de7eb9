#!/bin/bash
# k_mfma_ks with per-step records (no GCAP padding): ks parity tests, the headline bench, traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
mkdir -p gpurun_out/kspack
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread -k "ks or mfma or configs" > gpurun_out/kspack/tests.log 2>&1
tail -2 gpurun_out/kspack/tests.log
timeout -k 10 400 python3 bench.py --workload c5h > gpurun_out/kspack/c5h.json 2> gpurun_out/kspack/c5h.err
scripts/gpu_traffic_c5h.sh
