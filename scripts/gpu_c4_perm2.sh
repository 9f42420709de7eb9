#!/bin/bash
# com-Orkut: permutation variants (gather / scatter / hot-only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05i}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py -x -q -k "column_permutation" --timeout 120 --timeout-method thread > $OUT/pytest_perm.log 2>&1 || { tail -30 $OUT/pytest_perm.log; exit 1; }
tail -1 $OUT/pytest_perm.log
run() {
  local tag=$1; shift
  timeout -k 10 600 python3 -u bench.py --workload c4o --pipeline merge_path --p0 1024 --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse "$@" > $OUT/c4o_$tag.log 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/c4o_$tag.log') if l.startswith('{')][-1]
print('$tag', d['ms_per_step'], d['roofline']['frac'])"
}
run gather
run scatter --config MP_PERM_SCATTER=1
run hot256k --config MP_PERM_HOT=262144
run hot1m --config MP_PERM_HOT=1048576
echo done
