#!/bin/bash
# com-Orkut stand-in: merge_path(1024) with MP_COL_PARTS = 0 (one pass) / 4 / 8 column partitions
# (VERDICT r05 #2), one bench line each, GS_CONFIG holding the switch (EXTRA_CFG: more keys, e.g.
# ', "MP_GPF": 1').
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
set -e
for P in ${PARTS:-0 4 8}; do
  echo "{\"MP_COL_PARTS\": $P${EXTRA_CFG:-}}" > $OUT/cfg_$P.json
  GS_CONFIG=$OUT/cfg_$P.json timeout -k 10 600 python3 -u bench.py --workload c4o --pipeline merge_path --p0 1024 \
    --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS:-} > $OUT/c4o_parts$P.log 2>&1
  tail -1 $OUT/c4o_parts$P.log | cut -c1-400
done
