#!/bin/bash
# Round-3 quick GPU check: memory-floor probe, C4 (merge-path chain ordering), C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03q}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 120 scripts/probes/probe_floor > $OUT/probe_floor.txt 2>&1
for wl in ${WLS:-c4 c2}; do
  timeout -k 10 400 python3 bench.py --workload $wl --steps ${STEPS:-200} --warmup ${WARM:-50} --no-cpu > $OUT/bench_$wl.log 2>&1
  tail -1 $OUT/bench_$wl.log | cut -c1-200
done
echo quick done
