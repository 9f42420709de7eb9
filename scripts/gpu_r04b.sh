#!/bin/bash
# round 4: k_mfma_ks timelines at 40 / 80 rows, the pinned headline plans, smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04b
mkdir -p $OUT
EXP=$PWD/generalsparse_amd/libgeneralsparse_exp.so
GS_LIBRARY=$EXP timeout -k 10 120 python3 -u scripts/ks_timeline.py 40 > $OUT/tl40.json 2> $OUT/tl40.err
GS_LIBRARY=$EXP timeout -k 10 120 python3 -u scripts/ks_timeline.py 80 > $OUT/tl80.json 2> $OUT/tl80.err
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -m gpu -k "headline" > $OUT/pin.log 2>&1
tail -3 $OUT/pin.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
