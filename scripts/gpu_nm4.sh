#!/bin/bash
# k_nm_mfma4 (2:4 panels, 256-row workgroups, K split, B by LDS-DMA): parity, then C3 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05g}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nm.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_nm.log 2>&1 || { tail -30 $OUT/pytest_nm.log; exit 1; }
tail -1 $OUT/pytest_nm.log
run() {
  local tag=$1; shift
  timeout -k 10 400 python3 -u bench.py --workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse "$@" > $OUT/c3_$tag.log 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/c3_$tag.log') if l.startswith('{')][-1]
print('$tag', d['config']['kernel'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['hot_cache_kernel_ms'])"
}
run v4auto
run v4s1 --config NM_SPLIT=1
run v4s3 --config NM_SPLIT=3
run v4s4 --config NM_SPLIT=4
run classic --config NM_V4=0
echo done
