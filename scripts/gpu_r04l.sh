#!/bin/bash
# k_mfma_kb v2 (values staged through LDS): parity, C2 sweep, attribution
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04l
mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bm.py -x -q --timeout 120 --timeout-method thread -m gpu -k "kb" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SWEEP_KB=1 timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,48,64,80,96 0,2,4 8 > $OUT/sweep_kb.jsonl 2>&1
cat $OUT/sweep_kb.jsonl
for d in 2 3; do
  echo "GS_KB_DEBUG=$d" >> $OUT/dbg.jsonl
  GS_KB_DEBUG=$d SWEEP_KB=1 timeout -k 10 200 python3 -u scripts/ks_sweep_c2.py 40,96 0,4 8 >> $OUT/dbg.jsonl 2>&1
done
cat $OUT/dbg.jsonl
