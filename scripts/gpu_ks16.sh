#!/bin/bash
# k_mfma_ks with 16 waves (KS_WAVES=16): parity, then C2 and the headline layer against 8 waves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ks16}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 120 --timeout-method thread -k "mfma_ks" > $OUT/test.log 2>&1
tail -2 $OUT/test.log
timeout -k 10 300 python3 bench.py --workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --config KS_WAVES=16 > $OUT/c2.log 2>&1
tail -1 $OUT/c2.log | cut -c1-150
timeout -k 10 300 python3 bench.py --workload c5h --steps 100 --warmup 10 --no-cpu --no-rocsparse --config KS_WAVES=16 > $OUT/c5h.log 2>&1
tail -1 $OUT/c5h.log | cut -c1-150
echo ks16 done
