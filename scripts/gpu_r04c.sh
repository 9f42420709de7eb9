#!/bin/bash
# k_mfma_ks tagged-slab combine: parity, timelines, C2 sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "ks or headline or c5 or emitted" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
EXP=$PWD/generalsparse_amd/libgeneralsparse_exp.so
GS_LIBRARY=$EXP timeout -k 10 120 python3 -u scripts/ks_timeline.py 40 > $OUT/tl40.json 2> $OUT/tl40.err
GS_LIBRARY=$EXP timeout -k 10 120 python3 -u scripts/ks_timeline.py 80 > $OUT/tl80.json 2> $OUT/tl80.err
cat $OUT/tl40.json $OUT/tl80.json
timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,48,80 0 8 > $OUT/sweep.jsonl 2> $OUT/sweep.err
cat $OUT/sweep.jsonl
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "nm or c3" > $OUT/nm.log 2>&1 || { tail -30 $OUT/nm.log; exit 1; }
tail -2 $OUT/nm.log
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 50 --warmup 50 --no-rocsparse --no-cpu --n-sweep 8,32,128 > $OUT/c3.json 2> $OUT/c3.err
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().split(chr(10))[-1]); print(d['value'], d['roofline']['frac'], [(x['N'], x.get('kernel'), x.get('hbm_frac')) for x in d['n_sweep']])"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "merge or c4_web" > $OUT/mp.log 2>&1 || { tail -30 $OUT/mp.log; exit 1; }
tail -2 $OUT/mp.log
timeout -k 10 400 python3 -u bench.py --workload c4 --steps 50 --warmup 50 --no-rocsparse --no-cpu > $OUT/c4.json 2> $OUT/c4.err
python3 -c "import json; d=json.loads(open('$OUT/c4.json').read().strip().split(chr(10))[-1]); print(d['value'], d['roofline']['frac'], d['config']['plan'], {k: v.get('kernel_ms') for k, v in d['variants'].items()})"
