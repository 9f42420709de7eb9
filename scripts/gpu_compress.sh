#!/bin/bash
# Device index compression session: GPU parity tests of the formula
# path, the emitted programs (which pass the formulas too), then the traffic workload of
# scripts/compress_traffic.py with compression off / on: event timing, kernel stats and
# FETCH_SIZE / WRITE_SIZE passes.  Every GPU step has its own limit; any failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/compress
mkdir -p $OUT
export TMPDIR=/tmp
set -e
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_compress.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/tests.log 2>&1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -m gpu -k emitted > $OUT/emitted.log 2>&1
fi
for c in 0 1; do
  timeout -k 10 120 python3 scripts/compress_traffic.py $c 200 > $OUT/run$c.log 2>&1
  tail -1 $OUT/run$c.log
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$c -o prof -- python3 scripts/compress_traffic.py $c 100 > $OUT/prof$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc$c/fetch -o p -- python3 scripts/compress_traffic.py $c 20 > $OUT/fetch$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc$c/write -o p -- python3 scripts/compress_traffic.py $c 20 > $OUT/write$c.log 2>&1
done
echo "compress done"
