#!/bin/bash
# L2 hit rate (TCC_HIT / (TCC_HIT + TCC_MISS), MI355X_MICROARCH.md) and fabric read requests of the
# merge-path kernels on the C4 stand-ins: one PMC pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
set -e
for wl in ${WLS:-c4o c4}; do
  p0=1024; [ $wl = c4 ] && p0=256
  timeout -s KILL 500 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/l2_$wl -o p -- \
    python3 bench.py --workload $wl --pipeline merge_path --p0 $p0 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse \
    > $OUT/l2_$wl.log 2>&1
  echo "l2 $wl done"
done
