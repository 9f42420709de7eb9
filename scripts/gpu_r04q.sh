#!/bin/bash
# c5h with the layer-level attn choice (grouped attn launch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 700 python3 -u bench.py --workload c5h --steps 50 --warmup 20 > $OUT/c5h.json 2> $OUT/c5h.err
python3 -c "
import json; d=json.loads(open('$OUT/c5h.json').read().strip().split(chr(10))[-1]); print('c5h', d['value'], d['ms_per_step'], d['roofline']['frac'], d['serial_kernels']['hbm_frac'], d.get('speedup_vs_rocsparse')); print(d['layer_search'])
for k,v in d['per_shape'].items(): print(k, v['plan'], v['kernel'], v['kernel_us'], v['hbm_frac'])"
