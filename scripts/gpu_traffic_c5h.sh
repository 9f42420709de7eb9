#!/bin/bash
# PMC traffic per launch for every (shape, candidate) of the headline layer's plan search
# (separate FETCH_SIZE / WRITE_SIZE passes, one process each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
export TMPDIR=/tmp
rm -rf gpurun_out/tc5h; mkdir -p gpurun_out/tc5h
for sc in $(python3 scripts/traffic_c5h.py list); do
  s=${sc%%:*}; c=${sc##*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/tc5h/fetch_${s}_${c} -o p -- python3 scripts/traffic_c5h.py run $s $c 8 > gpurun_out/tc5h/fetch_${s}_${c}.log 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/tc5h/write_${s}_${c} -o p -- python3 scripts/traffic_c5h.py run $s $c 8 > gpurun_out/tc5h/write_${s}_${c}.log 2>&1
  echo "done $s $c"
done
python3 scripts/traffic_c5h.py summarize gpurun_out/tc5h 8 gpurun_out/tc5h/traffic_c5h.json
