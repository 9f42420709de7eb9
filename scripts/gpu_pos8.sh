#!/bin/bash
# 8-bit K-split entry positions (KS_POS8): parity, then C2 and the headline layer A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05h}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spmm.py -x -q -k "pos8 or mfma_ks or batch or four_waves" --timeout 200 --timeout-method thread > $OUT/pytest_p8.log 2>&1 || { tail -30 $OUT/pytest_p8.log; exit 1; }
tail -1 $OUT/pytest_p8.log
for cfg in "KS_POS8=0" "KS_POS8=1" "KS_WAVES=4" "KS_WAVES=4 --config KS_POS8=1"; do
  tag=$(echo $cfg | tr -c 'A-Za-z0-9=' '_')
  timeout -k 10 600 python3 -u bench.py --workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --config $cfg > $OUT/c2_$tag.log 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/c2_$tag.log') if l.startswith('{')][-1]
ns=d.get('north_star',{})
print('$cfg', d['config']['plan'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['hot_cache_kernel_ms'], 'layer', ns.get('ms_per_step'), ns.get('roofline',{}).get('frac'), ns.get('config',{}).get('launches_per_step'))"
done
echo done
