#!/bin/bash
# Round-3 GPU session: the -m gpu suite, smoke, then bench lines + rocprofv3 kernel stats per workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
  tail -3 $OUT/gputest.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -4 $OUT/smoke.log
fi
for wl in ${WLS:-c2 c1 c3 c4 c5 c5h}; do
  timeout -k 10 400 python3 bench.py --workload $wl --steps ${STEPS:-200} --warmup ${WARM:-50} > $OUT/bench_$wl.log 2>&1
  tail -1 $OUT/bench_$wl.log | cut -c1-240
  if [ -z "$NOPROF" ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o p -- python3 bench.py --workload $wl --steps 100 --warmup 20 --no-cpu --no-rocsparse > $OUT/prof_$wl.log 2>&1
  fi
done
echo r03 session done
