#!/bin/bash
# L2 hit rate and fabric read requests of com-Orkut's merge-path passes with MP_COL_PARTS = P
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
set -e
for P in ${PARTS:-4}; do
  echo "{\"MP_COL_PARTS\": $P}" > $OUT/cfg_$P.json
  GS_CONFIG=$OUT/cfg_$P.json timeout -s KILL 500 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
    -d $OUT/l2_p$P -o p -- python3 bench.py --workload c4o --pipeline merge_path --p0 1024 --steps 3 --warmup 1 --search-reps 2 \
    --search-rounds 1 --no-cpu --no-rocsparse > $OUT/l2_p$P.log 2>&1
  echo "l2 parts $P done"
done
