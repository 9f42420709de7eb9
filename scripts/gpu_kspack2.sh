#!/bin/bash
# k_mfma_ks records through vector loads: ks parity tests, headline layer and C5 batch bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
OUT=gpurun_out/kspack2
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread -k "ks or mfma or configs" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
timeout -k 10 400 python3 bench.py --workload c5h > $OUT/c5h.json 2> $OUT/c5h.err
tail -1 $OUT/c5h.json | cut -c1-200
timeout -k 10 500 python3 bench.py --workload c5 --steps 20 --warmup 20 > $OUT/c5.json 2> $OUT/c5.err
tail -1 $OUT/c5.json | cut -c1-200
