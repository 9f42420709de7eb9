#!/bin/bash
# 8-bit K-split entry positions (KS_POS8): parity, then C2 and the headline layer A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05h}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spmm.py -x -q -k "pos8 or mfma_ks or batch" --timeout 200 --timeout-method thread > $OUT/pytest_p8.log 2>&1 || { tail -30 $OUT/pytest_p8.log; exit 1; }
tail -1 $OUT/pytest_p8.log
for p8 in 0 1; do
  timeout -k 10 600 python3 -u bench.py --workload c2 --steps 200 --warmup 50 --no-cpu --config KS_POS8=$p8 > $OUT/c2_p8_$p8.log 2>&1
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/c2_p8_$p8.log') if l.startswith('{')][-1]
ns=d.get('north_star',{})
print('p8=$p8', d['config']['plan'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['hot_cache_kernel_ms'], 'layer', ns.get('ms_per_step'), ns.get('roofline',{}).get('frac'))"
done
echo done
