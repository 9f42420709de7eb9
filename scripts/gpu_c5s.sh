#!/bin/bash
# C5 / c5h with 1, 2, 3 streams (launch tails overlapped)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c5s}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
for st in 1 2 3; do
  timeout -k 10 300 python3 bench.py --workload c5h --steps 50 --warmup 10 --no-cpu --no-rocsparse --streams $st --search-reps 30 > $OUT/c5h_s$st.log 2>&1
  tail -1 $OUT/c5h_s$st.log | cut -c1-160
done
for st in 1 2; do
  timeout -k 10 400 python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu --no-rocsparse --streams $st --search-reps 30 > $OUT/c5_s$st.log 2>&1
  tail -1 $OUT/c5_s$st.log | cut -c1-160
done
for wl in c2 c3 c4; do
  timeout -k 10 400 python3 bench.py --workload $wl --steps 50 --warmup 10 --no-cpu --no-rocsparse --search-reps 40 --n-sweep 8,32,128 > $OUT/nsweep_$wl.log 2>&1
  tail -1 $OUT/nsweep_$wl.log | cut -c1-100
done
echo c5s done
