#!/bin/bash
# grouped k_mfma_ks launches: parity, headline layer and C5 batch grouped vs per-matrix launches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "batch or ks or headline or c5 or emitted" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for G in 1; do
timeout -k 10 600 python3 -u bench.py --workload c5h --steps 20 --warmup 10 --no-rocsparse --group $G > $OUT/c5h_g$G.json 2> $OUT/c5h_g$G.err
python3 -c "
import json; d=json.loads(open('$OUT/c5h_g$G.json').read().strip().split(chr(10))[-1]); print('c5h group=$G', d['value'], d['ms_per_step'], d['roofline']['frac'], d['serial_kernels']['hbm_frac'])"
done
for G in 1; do
timeout -k 10 900 python3 -u bench.py --workload c5 --steps 10 --warmup 5 --group $G > $OUT/c5_g$G.json 2> $OUT/c5_g$G.err
python3 -c "
import json; d=json.loads(open('$OUT/c5_g$G.json').read().strip().split(chr(10))[-1]); print('c5 group=$G', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
