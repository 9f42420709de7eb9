#!/bin/bash
# Round-2 bench lines of every BASELINE config + rocprofv3 kernel stats (profiles/r02_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
for wl in ${WLS:-c2 c1 c3 c4 c5}; do
  timeout -k 10 400 python3 bench.py --workload $wl --steps ${STEPS:-200} --warmup ${WARM:-50} > $OUT/bench_$wl.log 2>&1
  tail -1 $OUT/bench_$wl.log | cut -c1-200
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o p -- python3 bench.py --workload $wl --steps 100 --warmup 20 --no-cpu --no-rocsparse > $OUT/prof_$wl.log 2>&1
done
echo r02 bench done
