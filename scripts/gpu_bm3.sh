#!/bin/bash
# k_mfma_bm2 bring-up: parity (bm and bm2), C2 bench with MFMA_BM=1 (bm2) and BM_V2=0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bm3}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bm.py -x -q --timeout 120 --timeout-method thread > $OUT/test_bm.log 2>&1
tail -2 $OUT/test_bm.log
timeout -k 10 300 python3 bench.py --workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --config MFMA_BM=1 > $OUT/bench_c2_bm2.log 2>&1
tail -1 $OUT/bench_c2_bm2.log | cut -c1-200
echo bm3 done
