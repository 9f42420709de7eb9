#!/bin/bash
# k_mfma_ks step claiming + last-wave ticket: parity, timelines, C2 sweep, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "ks or headline or c5 or emitted" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
EXP=$PWD/generalsparse_amd/libgeneralsparse_exp.so
GS_LIBRARY=$EXP timeout -k 10 120 python3 -u scripts/ks_timeline.py 40 > $OUT/tl40.json 2> $OUT/tl40.err
GS_LIBRARY=$EXP timeout -k 10 120 python3 -u scripts/ks_timeline.py 80 > $OUT/tl80.json 2> $OUT/tl80.err
GS_LIBRARY=$EXP KS_OLD_SHARE=40 timeout -k 10 120 python3 -u scripts/ks_timeline.py 40 > $OUT/tl40s40.json 2> $OUT/tl40s40.err
cat $OUT/tl40.json $OUT/tl80.json $OUT/tl40s40.json
SWEEP_SHARE=32,36,40 timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,80 0 8 > $OUT/share.jsonl 2>&1; cat $OUT/share.jsonl
timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 48,64,96,112,128 0 8 > $OUT/sweep.jsonl 2> $OUT/sweep.err
cat $OUT/sweep.jsonl
timeout -k 10 400 python3 -u bench.py --steps 100 --warmup 200 --no-rocsparse --no-cpu > $OUT/c2.json 2> $OUT/c2.err
python3 -c "import json; d=json.loads(open('$OUT/c2.json').read().strip().split(chr(10))[-1]); print(d['value'], d['roofline']['frac'], d['config']['plan'], {k: v.get('kernel_ms') for k, v in d['variants'].items()})"
timeout -k 10 600 python3 -u bench.py --workload c5h --steps 20 --warmup 10 --no-rocsparse > $OUT/c5h.json 2> $OUT/c5h.err
python3 -c "
import json; d=json.loads(open('$OUT/c5h.json').read().strip().split(chr(10))[-1]); print('c5h', d['value'], d['roofline']['frac'], d['serial_kernels'])
for k,v in d['per_shape'].items(): print(k, v['plan'], v['kernel'], v['kernel_us'], v['hbm_frac'], {a: b.get('kernel_us') for a, b in v['variants'].items()})"
