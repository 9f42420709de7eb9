#!/bin/bash
# Round-3 final-tree session: -m gpu suite + smoke (PART=a), bench lines + rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03b}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
if [ "$PART" = "a" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
  tail -2 $OUT/gputest.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -4 $OUT/smoke.log
fi
for wl in $WLS; do
  steps=200; psteps=100
  if [ "$wl" = "c5" ]; then steps=20; psteps=5; fi
  timeout -k 10 500 python3 bench.py --workload $wl --steps $steps --warmup 20 > $OUT/bench_$wl.log 2>&1
  tail -1 $OUT/bench_$wl.log | cut -c1-200
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o p -- python3 bench.py --workload $wl --steps $psteps --warmup 10 --no-cpu --no-rocsparse > $OUT/prof_$wl.log 2>&1
done
echo r03b $PART done
