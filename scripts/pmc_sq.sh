#!/bin/bash
# SQ/LDS PMC passes on one plan (separate runs, --kernel-trace only).
# usage: pmc_sq.sh TAG args...   (PROG = profiled script, default scripts/prof_one.py
# with args: pipeline p0 p1 dtype N)
PROG=${PROG:-scripts/prof_one.py}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-lds}; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- python3 $PROG "$@" > $OUT/trace.log 2>&1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o p -- python3 $PROG "$@" > $OUT/p$i.log 2>&1
done
echo pmc done
