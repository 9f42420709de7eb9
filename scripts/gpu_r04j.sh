#!/bin/bash
# k_mfma_kb (k_mfma_ks pipeline on the bitmap layout, experiments build): parity, then the C2 sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04j
mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bm.py -x -q --timeout 120 --timeout-method thread -m gpu -k "kb" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SWEEP_KB=1 timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,48,64,80,96 0,2,4,8 8 > $OUT/sweep_kb.jsonl 2>&1
cat $OUT/sweep_kb.jsonl
timeout -k 10 200 python3 -u scripts/ks_sweep_c2.py 40,80 0 8 > $OUT/sweep_ks.jsonl 2>&1
cat $OUT/sweep_ks.jsonl
