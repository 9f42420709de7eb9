#!/bin/bash
# k_mfma_bm timeline on C2 (80- and 96-row blocks) + variant sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bm2}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 120 python3 scripts/bm_timeline.py 80 > $OUT/timeline80.json 2>&1
cat $OUT/timeline80.json | tail -1
timeout -k 10 300 python3 bench.py --workload c2 --steps 100 --warmup 20 --no-cpu --no-rocsparse --config MFMA_BM=1 --config BM_WAVES=4 > $OUT/bench_c2_w4.log 2>&1
timeout -k 10 300 python3 bench.py --workload c2 --steps 100 --warmup 20 --no-cpu --no-rocsparse --config MFMA_BM=1 --config BM_SPLIT=8 > $OUT/bench_c2_s8.log 2>&1
echo bm2 done
