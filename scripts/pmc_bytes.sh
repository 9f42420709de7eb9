#!/bin/bash
# Request-size-resolved L2 <-> fabric traffic of one bench workload (separate
# B-row gather over-fetch from A streaming).  Two counter passes (<= 4 TCC each) plus the
# kernel stats; summarised by scripts/pmc_bytes.py.  usage: WL=c4 [PIPE=merge_path P0=512] pmc_bytes.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WL=${WL:-c4}
OUT=gpurun_out/bytes_$WL
mkdir -p $OUT
export TMPDIR=/tmp
set -e
ARGS="--workload $WL --steps 20 --warmup 2 --no-cpu --no-rocsparse --search-reps 5"
[ -n "$PIPE" ] && ARGS="$ARGS --pipeline $PIPE --p0 $P0 --p1 ${P1:-1}"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_BUBBLE_sum --output-format csv -d $OUT/p1 -o p -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $OUT/p2 -o p -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/p3 -o p -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
echo "$WL bytes done"
