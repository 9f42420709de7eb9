#!/bin/bash
# C4 (BASELINE.json configs[3], webbase-1M stand-in) session: merge-path GPU
# tests, bench line, rocprofv3 kernel stats of the merge-path plan, FETCH_SIZE /
# WRITE_SIZE passes.  Every GPU step has its own limit; any failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WL=${WL:-c4}
OUT=gpurun_out/$WL
mkdir -p $OUT
export TMPDIR=/tmp
set -e
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 120 --timeout-method thread -m gpu -k "merge or balanced" > $OUT/tests.log 2>&1
fi
timeout -k 10 600 python3 bench.py --workload $WL --steps ${STEPS:-100} --warmup 10 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log
P0=${P0:-1024}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --workload $WL --pipeline merge_path --p0 $P0 --steps ${STEPS:-100} --warmup 10 --no-cpu --no-rocsparse > $OUT/prof.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o p -- python3 bench.py --workload $WL --pipeline merge_path --p0 $P0 --steps 20 --warmup 2 --no-cpu --no-rocsparse > $OUT/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o p -- python3 bench.py --workload $WL --pipeline merge_path --p0 $P0 --steps 20 --warmup 2 --no-cpu --no-rocsparse > $OUT/write.log 2>&1
echo "$WL done"
