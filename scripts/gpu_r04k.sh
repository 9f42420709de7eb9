#!/bin/bash
# k_mfma_kb attribution (experiments build, GS_KB_DEBUG builds give wrong results): full,
# 8-B-aligned windows, no windows, no B loads; 40-row (S 2) and 96-row (S 4) blocks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04k
mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
for d in 0 1 2 3; do
  echo "GS_KB_DEBUG=$d" >> $OUT/sweep.jsonl
  GS_KB_DEBUG=$d SWEEP_KB=1 timeout -k 10 200 python3 -u scripts/ks_sweep_c2.py 40,96 0,4 8 >> $OUT/sweep.jsonl 2>&1
done
cat $OUT/sweep.jsonl
# k_mfma_ks phase timelines: C2 40-row, attn (7168^2) 56-row
timeout -k 10 120 python3 -u scripts/ks_timeline.py 40 > $OUT/tl_c2_40.json 2>&1
TL_M=7168 timeout -k 10 120 python3 -u scripts/ks_timeline.py 56 > $OUT/tl_attn_56.json 2>&1
cat $OUT/tl_c2_40.json $OUT/tl_attn_56.json
