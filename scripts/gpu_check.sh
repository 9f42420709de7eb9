#!/bin/bash
# GPU suite + smoke + default bench line (one call); stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/check
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -2 $OUT/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20} > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-600
