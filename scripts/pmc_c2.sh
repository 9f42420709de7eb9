#!/bin/bash
# PMC passes (separate runs, --kernel-trace only, per MI355X_MICROARCH.md) on the bench's best plan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-r01}
mkdir -p $OUT
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 bench.py --steps 50 --warmup 5 --pipeline tblock_warp_total --no-cpu --no-rocsparse > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 bench.py --steps 50 --warmup 5 --pipeline tblock_warp_total --no-cpu --no-rocsparse > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d $OUT/tcc -o p -- python3 bench.py --steps 50 --warmup 5 --pipeline tblock_warp_total --no-cpu --no-rocsparse > $OUT/tcc.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/tcp -o p -- python3 bench.py --steps 50 --warmup 5 --pipeline tblock_warp_total --no-cpu --no-rocsparse > $OUT/tcp.log 2>&1
echo pmc done
