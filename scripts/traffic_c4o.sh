#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md HBM section) of the com-Orkut
# stand-in on merge_path(2048) and on merge_path(1024) with MP_COL_PARTS=4; summed per launch by
# scripts/traffic_c4o.py into profiles/traffic_c4o.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06fin}
OUT=gpurun_out/$TAG/tc4o
mkdir -p $OUT
set -e
echo '{"MP_COL_PARTS": 0}' > $OUT/cfg_p0.json
echo '{"MP_COL_PARTS": 4}' > $OUT/cfg_p4.json
for v in "p0 2048" "p4 1024"; do
  set -- $v
  for c in FETCH_SIZE WRITE_SIZE; do
    GS_CONFIG=$OUT/cfg_$1.json timeout -s KILL 500 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$1_$c -o p -- \
      python3 bench.py --workload c4o --pipeline merge_path --p0 $2 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 \
      --no-cpu --no-rocsparse > $OUT/$1_$c.log 2>&1
    echo "$1 $c done"
  done
done
