#!/bin/bash
# C5 batch: GPU tests of the shapes/batch, bench line, rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c5
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k c5 -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 500 python3 bench.py --workload c5 --steps ${STEPS:-20} --warmup ${WARM:-5} > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-900
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 bench.py --workload c5 --steps 10 --warmup 3 > $OUT/prof.log 2>&1
echo c5 done
