#!/bin/bash
# k_mfma_ks look-ahead depth sweep (experiments build, GS_KS_DEPTH): C2 40-row, attn 56-row,
# fc1 / fc2 112-row
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04n
mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
for d in 0 2 3 6; do
  GS_KS_DEPTH=$d timeout -k 10 120 python3 -u scripts/ks_sweep_c2.py 40 0 8 >> $OUT/c2.jsonl 2>&1
  GS_KS_DEPTH=$d timeout -k 10 200 python3 -u scripts/shape_time.py attn 1 >> $OUT/shapes.jsonl 2>&1
  GS_KS_DEPTH=$d timeout -k 10 200 python3 -u scripts/shape_time.py fc1 4 >> $OUT/shapes.jsonl 2>&1
done
grep -v amdgpu.ids $OUT/c2.jsonl $OUT/shapes.jsonl
