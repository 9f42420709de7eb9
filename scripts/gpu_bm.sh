#!/bin/bash
# k_mfma_bm bring-up: unaligned-load probe, bm parity tests, C2 bench with MFMA_BM on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bm}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 60 scripts/probes/probe_unaligned > $OUT/probe_unaligned.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bm.py -x -q --timeout 120 --timeout-method thread > $OUT/test_bm.log 2>&1
tail -2 $OUT/test_bm.log
timeout -k 10 300 python3 bench.py --workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --config MFMA_BM=1 > $OUT/bench_c2_bm.log 2>&1
tail -1 $OUT/bench_c2_bm.log | cut -c1-300
timeout -k 10 120 scripts/probes/probe_floor > $OUT/probe_floor.txt 2>&1
timeout -k 10 300 python3 bench.py --workload c4 --steps 200 --warmup 50 --no-cpu --no-rocsparse > $OUT/bench_c4.log 2>&1
tail -1 $OUT/bench_c4.log | cut -c1-200
echo bm done
