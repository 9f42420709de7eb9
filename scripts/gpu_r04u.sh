#!/bin/bash
# alternating-epoch slab tags (no slab clearing): parity (ks, headline, batch, nm, emitted; kb in
# the experiments build), C2 / c5h bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04u
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py tests/test_gpu_nm.py -x -q --timeout 300 --timeout-method thread -m gpu -k "ks or headline or batch or nm or emitted or c5 or c3" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bm.py -x -q --timeout 120 --timeout-method thread -m gpu -k "kb" > $OUT/tests_kb.log 2>&1 || { tail -30 $OUT/tests_kb.log; exit 1; }
tail -1 $OUT/tests_kb.log
timeout -k 10 500 python3 -u bench.py --steps 200 --warmup 20 > $OUT/c2.json 2> $OUT/c2.err
python3 -c "import json; d=json.loads(open('$OUT/c2.json').read().strip().split(chr(10))[-1]); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config']['plan'])"
timeout -k 10 700 python3 -u bench.py --workload c5h --steps 50 --warmup 20 > $OUT/c5h.json 2> $OUT/c5h.err
python3 -c "
import json; d=json.loads(open('$OUT/c5h.json').read().strip().split(chr(10))[-1]); print('c5h', d['value'], d['ms_per_step'], d['roofline']['frac'], d['serial_kernels']['hbm_frac']); print(d['layer_search'])
for k,v in d['per_shape'].items(): print(k, v['plan'], v['kernel'], v['kernel_us'], v['hbm_frac'])"
