#!/bin/bash
# scratch GPU step: A/B vs the previous build, full GPU suite, compression traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/step
export TMPDIR=/tmp
set -e
bash scripts/gpu_ab.sh
timeout -k 10 1000 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/step/tests.log 2>&1
tail -2 gpurun_out/step/tests.log
SKIP_TESTS=1 bash scripts/gpu_compress.sh
