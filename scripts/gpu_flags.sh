#!/bin/bash
# k_mfma_rows with LDS counter hand-offs (MFMA_FLAGS): parity, then C2 / c5h against barriers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-flags}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 120 --timeout-method thread -k counter_handoffs > $OUT/test_flags.log 2>&1
tail -2 $OUT/test_flags.log
timeout -k 10 300 python3 bench.py --workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --config MFMA_FLAGS=1 > $OUT/bench_c2_flags.log 2>&1
tail -1 $OUT/bench_c2_flags.log | cut -c1-200
timeout -k 10 300 python3 bench.py --workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse > $OUT/bench_c2.log 2>&1
tail -1 $OUT/bench_c2.log | cut -c1-200
echo flags done
