#!/bin/bash
# LDS counters (bank-conflict cycles, LDS-array cycles, LDS instructions) of the C2 / C3 bench
# kernels, one rocprofv3 --pmc pass per workload (scripts/session_params.sh pmc_cmd).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/session_params.sh
TAG=${TAG:-r05lds}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
set -e
for wl in ${WLS:-c2 c3}; do
  cmd=$(pmc_cmd $wl)
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/lds_$wl -o p -- $cmd > $OUT/lds_$wl.log 2>&1
  echo "lds $wl done"
done
