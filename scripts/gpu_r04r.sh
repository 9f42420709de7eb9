#!/bin/bash
# KS_PRIO 0 / 1 / 2 at look-ahead 2; D 1 vs 2 on the 112-row plans (experiments build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04r
mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
for pr in 0 1 2; do
  SWEEP_PRIO=$pr timeout -k 10 120 python3 -u scripts/ks_sweep_c2.py 40 0 8 >> $OUT/c2.jsonl 2>&1
  for sc in "attn 4" "fc1 4" "fc2 4"; do
    SWEEP_CFG=KS_PRIO=$pr timeout -k 10 200 python3 -u scripts/shape_time.py $sc >> $OUT/shapes.jsonl 2>&1
  done
done
for sc in "attn 4" "fc1 4" "fc2 4"; do
  GS_KS_DEPTH=1 timeout -k 10 200 python3 -u scripts/shape_time.py $sc >> $OUT/shapes.jsonl 2>&1
done
grep -v amdgpu.ids $OUT/c2.jsonl $OUT/shapes.jsonl
