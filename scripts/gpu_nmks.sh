#!/bin/bash
# k_nm_mfma_ks bring-up: 2:4 parity tests, emitted programs, C3 bench (+ classic kernel for comparison)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-nmks}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nm.py -x -q --timeout 120 --timeout-method thread > $OUT/test_nm.log 2>&1
tail -2 $OUT/test_nm.log
timeout -k 10 300 python3 bench.py --workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-200
timeout -k 10 300 python3 bench.py --workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse --config NM_KS=0 > $OUT/bench_c3_classic.log 2>&1
tail -1 $OUT/bench_c3_classic.log | cut -c1-200
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -k "emitted or c3" > $OUT/test_cfg.log 2>&1
tail -2 $OUT/test_cfg.log
echo nmks done
