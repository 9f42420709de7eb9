#!/bin/bash
# SQ / LDS PMC passes on k_mfma_ks (C2 40-row; fc1 112-row) and k_mfma_rows (attn 28-row)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
bash scripts/pmc_sq.sh ks_c2_40 block_total 40 1 f16 32 100
python3 scripts/pmc_summary.py gpurun_out/pmc_ks_c2_40 k_mfma > gpurun_out/pmc_ks_c2_40/summary.txt
PROG=scripts/traffic_c5h.py bash scripts/pmc_sq.sh ks_fc1_112 run fc1 4 30
python3 scripts/pmc_summary.py gpurun_out/pmc_ks_fc1_112 k_mfma > gpurun_out/pmc_ks_fc1_112/summary.txt
PROG=scripts/traffic_c5h.py bash scripts/pmc_sq.sh rows_attn_28 run attn 0 30
python3 scripts/pmc_summary.py gpurun_out/pmc_rows_attn_28 k_mfma > gpurun_out/pmc_rows_attn_28/summary.txt
cat gpurun_out/pmc_*/summary.txt
