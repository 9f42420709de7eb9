#!/bin/bash
# k_mfma_ks look-ahead depth sweep 2 (GS_KS_DEPTH 1/2/3 vs 4): C2 40 / 80-row, attn 56 / 112,
# fc1 / fc2 112-row
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04o
mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
for d in 0 1 2 3; do
  GS_KS_DEPTH=$d timeout -k 10 120 python3 -u scripts/ks_sweep_c2.py 40,80 0 8 | sed "s/^/D$d /" >> $OUT/c2.jsonl 2>&1
  for sc in "attn 1" "attn 4" "fc1 4" "fc2 4"; do
    GS_KS_DEPTH=$d timeout -k 10 200 python3 -u scripts/shape_time.py $sc >> $OUT/shapes.jsonl 2>&1
  done
done
grep -v amdgpu.ids $OUT/c2.jsonl $OUT/shapes.jsonl
