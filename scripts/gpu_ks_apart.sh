#!/bin/bash
# KS_APART A/B on C2: apart vs overlapped LDS layouts, K splits 2/4/8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05e}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py -x -q -k "overlapped or known_answer_and_c2 or driver_plan" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {
  local tag=$1; shift
  timeout -k 10 300 python3 -u bench.py --workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --no-north-star "$@" > $OUT/c2_$tag.log 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/c2_$tag.log') if l.startswith('{')][-1]
print('$tag', d['config']['plan'], d['config']['kernel'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['hot_cache_kernel_ms'])"
}
run base --pipeline block_total --p0 40
run ap0_s2 --pipeline block_total --p0 40 --config KS_APART=0
run ap0_s4 --pipeline block_total --p0 40 --config KS_APART=0 --config KS_SPLIT=4
run ap1_s4 --pipeline block_total --p0 40 --config KS_SPLIT=4
run ap0_80s4 --pipeline block_total --p0 80 --config KS_APART=0
run ap0_80s8 --pipeline block_total --p0 80 --config KS_APART=0 --config KS_SPLIT=8
run ap0_64s4 --pipeline block_total --p0 64 --config KS_APART=0 --config KS_SPLIT=4
run ap0_48s4 --pipeline block_total --p0 48 --config KS_APART=0 --config KS_SPLIT=4
echo done
