#!/bin/bash
# One GPU-box session (replaces the per-round scripts/gpu_r0*.sh one-offs, which live on in
# git history).  Usage: TAG=r05a PARTS="tests bench prof" WLS="c2 c5h" scripts/gpu_session.sh
# Parts (any subset, run in this order):
#   tests   the -m gpu suite, then smoke()
#   bench   one bench line per workload in $WLS (steps / warm-up from scripts/session_params.sh)
#   prof    rocprofv3 --kernel-trace --stats of the same bench command, per workload
#   pmc     FETCH_SIZE / WRITE_SIZE passes per workload in $PMC_WLS (traffic_<wl>.json)
#   sq      SQ / GRBM passes (MFMA utilisation) per workload in $PMC_WLS
# Every GPU step runs under its own time limit; the first failing step ends the session
# (set -e), so nothing else touches the GPU after a fault, abort or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/session_params.sh
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
set -e
has() { [[ " $PARTS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -8 $OUT/smoke.log
fi
for wl in $WLS; do
  steps=$(bench_steps $wl); psteps=$(prof_steps $wl)
  if has bench; then
    timeout -k 10 900 python3 -u bench.py --workload $wl --steps $steps --warmup 20 ${BENCH_ARGS:-} > $OUT/bench_$wl.log 2>&1
    tail -1 $OUT/bench_$wl.log | cut -c1-300
  fi
  if has prof; then
    # GS_BENCH_MARK=1: spin-kernel markers around the timed region, so timed_stats.py keeps only its dispatches
    GS_BENCH_MARK=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o p -- \
      python3 bench.py --workload $wl --steps $psteps --warmup 10 --no-cpu --no-rocsparse ${BENCH_ARGS:-} > $OUT/prof_$wl.log 2>&1
    python3 scripts/timed_stats.py $OUT/prof_$wl $OUT/prof_${wl}_timed_stats.csv > /dev/null || echo "timed_stats $wl: no marked region"
    echo "prof $wl done"
  fi
done
for wl in ${PMC_WLS:-}; do
  cmd=$(pmc_cmd $wl)
  if has pmc; then
    mkdir -p $OUT/pmc_$wl
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 600 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/pmc_$wl/$c -o p -- $cmd \
        > $OUT/pmc_$wl/$c.log 2>&1 || { echo "pmc $wl $c failed"; exit 1; }
    done
    echo "pmc $wl done"
  fi
  if has sq; then
    timeout -s KILL 600 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
      --output-format csv -d $OUT/sq_$wl -o p -- $cmd > $OUT/sq_$wl.log 2>&1
    echo "sq $wl done"
  fi
done
echo "session $TAG done"
