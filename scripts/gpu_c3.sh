#!/bin/bash
# C3 (BASELINE.json configs[2]) measurement session: bench line, rocprofv3
# kernel stats of the same command, FETCH_SIZE / WRITE_SIZE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c3
mkdir -p $OUT
export TMPDIR=/tmp
set -e
timeout -k 10 600 python3 bench.py --workload c3 --steps ${STEPS:-100} --warmup 10 > $OUT/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --workload c3 --steps ${STEPS:-100} --warmup 10 --no-cpu --no-rocsparse > $OUT/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o p -- python3 scripts/time_nm.py 28672 7168 128 30 > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o p -- python3 scripts/time_nm.py 28672 7168 128 30 > $OUT/write.log 2>&1
tail -1 $OUT/bench.log
echo c3 done
