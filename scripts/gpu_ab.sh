#!/bin/bash
# A/B of library builds on the same box: GS_LIBRARY=<pkg>/libgeneralsparse_<v>.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
set -e
for rep in 1 2; do
for v in ${LIBS:-main}; do
  [ "$v" = main ] && v=""
  for wl in ${WLS:-c1 c4}; do
    GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse$v.so timeout -k 10 300 python3 bench.py --workload $wl --steps 100 --warmup 10 --no-cpu --no-rocsparse > gpurun_out/ab/b${v}_$wl.log 2>&1
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab/b${v}_$wl.log') if l.startswith('{')][-1]
print('lib$v', '$wl', d['value'], d['roofline']['kernel_ms'], d['roofline']['hot_cache_kernel_ms'], d['config']['plan'])"
  done
done
done
