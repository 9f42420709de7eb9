#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats and
# the HBM-traffic PMC passes of the bench's best plan.
# Every GPU step has its own time limit; a fault/abort/timeout (exit >= 124 or
# 134/139) ends the session, an ordinary test failure (exit 1) does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-200}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || [ "$rc" -eq 5 ]; }
step() {
  local name=$1; shift
  echo "== $name: $*" | tee -a $OUT/session.log
  "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name exit $rc" | tee -a $OUT/session.log
  tail -3 $OUT/$name.log
  ok $rc || { echo "stopping after $name (exit $rc)"; exit $rc; }
}
rocm-smi --showproductname > $OUT/rocm_smi.log 2>&1 || true
nproc > $OUT/nproc.log; lscpu | grep -E "Model name|^CPU\(s\)" >> $OUT/nproc.log || true
[ -n "$SKIP_TESTS" ] || step pytest_gpu timeout -k 10 900 python -m pytest tests -m gpu -q
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 600 python bench.py --steps $STEPS --warmup 20
export TMPDIR=/tmp
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- python3 bench.py --steps $STEPS --warmup 20 --no-cpu --no-rocsparse
BEST=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/bench.log') if l.startswith('{')][-1]
n,a=d['config']['plan'].split('('); a=a.rstrip(')').split(','); print(n,a[0],a[1])" 2>/dev/null || echo "block_total 20 1")
step pmc_fetch timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/fetch -o p -- python3 scripts/prof_one.py $BEST f16 32 100
step pmc_write timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/write -o p -- python3 scripts/prof_one.py $BEST f16 32 100
echo "session done"
