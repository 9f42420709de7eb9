#!/bin/bash
# C4 merge-path timing probes (diagnostic): plan variants and GS_MP_DEBUG bits
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c4probe
mkdir -p $OUT
set -e
for p0 in ${P0S:-256 1024}; do
  for dbg in ${DBGS:-0 2}; do
    GS_MP_DEBUG=$dbg timeout -k 10 120 python3 bench.py --workload ${WL:-c4} --pipeline merge_path --p0 $p0 --steps 50 --warmup 5 --no-cpu --no-rocsparse > $OUT/p${p0}_d${dbg}.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$OUT/p${p0}_d${dbg}.log').read().strip().split('\n')[-1]); print('p0=$p0 dbg=$dbg', d['roofline']['kernel_ms'])"
  done
done
