#!/bin/bash
# C5 batch: per-matrix launches over two streams vs grouped launches (largest first) on 1 / 2 streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04s
mkdir -p $OUT
for cfg in "0 2" "1 1" "1 2"; do
  set -- $cfg
  timeout -k 10 600 python3 -u bench.py --workload c5 --steps 20 --warmup 10 --group $1 --streams $2 > $OUT/c5_g$1_s$2.json 2> $OUT/c5_g$1_s$2.err
  python3 -c "
import json; d=json.loads(open('$OUT/c5_g$1_s$2.json').read().strip().split(chr(10))[-1]); print('group $1 streams $2', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['plan'], v['kernel_us']) for k, v in d['per_shape'].items()})"
done
