#!/bin/bash
# com-Orkut stand-in: merge_path(1024) with MP_COL_PARTS=2 and MP_HUB_COLS = H (hub / tail
# column passes), one bench line per H, then a kernel trace of the first H (per-pass times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
set -e
for H in ${HUBS:-131072 65536}; do
  echo "{\"MP_COL_PARTS\": 2, \"MP_HUB_COLS\": $H}" > $OUT/cfg_$H.json
  GS_CONFIG=$OUT/cfg_$H.json timeout -k 10 600 python3 -u bench.py --workload c4o --pipeline merge_path --p0 ${P0:-1024} \
    --steps 20 --warmup 5 --no-cpu --no-rocsparse > $OUT/c4o_hub$H.log 2>&1
  tail -1 $OUT/c4o_hub$H.log | cut -c1-300
done
H=$(echo ${HUBS:-131072 65536} | cut -d' ' -f1)
GS_CONFIG=$OUT/cfg_$H.json timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$H -o p -- \
  python3 bench.py --workload c4o --pipeline merge_path --p0 ${P0:-1024} --steps 5 --warmup 2 --no-cpu --no-rocsparse > $OUT/trace_$H.log 2>&1
echo trace done
