#!/bin/bash
# k_mfma_ks younger-half priority (KS_PRIO 0/1/2): C2 sweep + timelines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04h
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 300 --timeout-method thread -m gpu -k "mfma_ks_known or batch" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SWEEP_PRIO=0,1,2 timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,80,112 0 8 > $OUT/sweep.jsonl 2> $OUT/sweep.err
cat $OUT/sweep.jsonl
EXP=$PWD/generalsparse_amd/libgeneralsparse_exp.so
for P in 1 2; do
GS_LIBRARY=$EXP KS_PRIO=$P timeout -k 10 120 python3 -u scripts/ks_timeline.py 40 > $OUT/tl40_p$P.json 2> $OUT/tl40_p$P.err
python3 -c "import json; d=json.load(open('$OUT/tl40_p$P.json')); print($P, d['loop_done_by_wave'], d['wg_span_clk'])"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nm.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "nm or c3 or emitted" > $OUT/nm.log 2>&1 || { tail -30 $OUT/nm.log; exit 1; }
tail -1 $OUT/nm.log
for T in 8 7; do
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 100 --warmup 50 --no-rocsparse --no-cpu --config NM_TPW=$T > $OUT/c3_t$T.json 2> $OUT/c3_t$T.err
python3 -c "import json; d=json.loads(open('$OUT/c3_t$T.json').read().strip().split(chr(10))[-1]); print('c3 tpw=$T', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
