#!/bin/bash
# interleaved k_mfma_ks (bc36caa body) + 96..128-row blocks: parity, C2, headline layer, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04e
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "ks or headline or c5 or emitted" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,80,112 0 8 > $OUT/sweep.jsonl 2> $OUT/sweep.err
cat $OUT/sweep.jsonl
timeout -k 10 600 python3 -u bench.py --workload c5h --steps 20 --warmup 10 > $OUT/c5h.json 2> $OUT/c5h.err
python3 -c "
import json; d=json.loads(open('$OUT/c5h.json').read().strip().split(chr(10))[-1]); print('c5h', d['value'], d['roofline']['frac'], d['serial_kernels'], d.get('speedup_vs_rocsparse'))
for k,v in d['per_shape'].items(): print(k, v['plan'], v['kernel'], v['kernel_us'], v['hbm_frac'], {a: b.get('kernel_us') for a, b in v['variants'].items()})"
timeout -k 10 900 python3 -u bench.py --workload c5 --steps 10 --warmup 5 > $OUT/c5.json 2> $OUT/c5.err
python3 -c "
import json; d=json.loads(open('$OUT/c5.json').read().strip().split(chr(10))[-1]); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['per_shape'])"
