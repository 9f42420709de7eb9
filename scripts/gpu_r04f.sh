#!/bin/bash
# merge-path phase timeline (C4) and the C2 dense-width sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04f
mkdir -p $OUT
EXP=$PWD/generalsparse_amd/libgeneralsparse_exp.so
GS_LIBRARY=$EXP timeout -k 10 200 python3 -u scripts/mp_timeline.py 512 > $OUT/mp512.json 2> $OUT/mp512.err
GS_LIBRARY=$EXP timeout -k 10 200 python3 -u scripts/mp_timeline.py 2048 > $OUT/mp2048.json 2> $OUT/mp2048.err
cat $OUT/mp512.json $OUT/mp2048.json
timeout -k 10 600 python3 -u bench.py --steps 50 --warmup 100 --no-rocsparse --no-cpu --n-sweep 8,32,128 --search-rounds 1 > $OUT/c2n.json 2> $OUT/c2n.err
python3 -c "import json; d=json.loads(open('$OUT/c2n.json').read().strip().split(chr(10))[-1]); print([(x['N'], x.get('plan'), x.get('kernel'), x.get('kernel_ms'), x.get('hbm_frac')) for x in d['n_sweep']])"
