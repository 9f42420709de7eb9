#!/bin/bash
# k_mfma_ks 128-column tiles: parity at N = 128 (and around), C2 dense-width sweep, DRAM-request split of com-Orkut
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05d}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_spmm.py -x -q -k "mfma_ks or slab or c2" --timeout 200 --timeout-method thread > $OUT/pytest_ks.log 2>&1 || { tail -30 $OUT/pytest_ks.log; exit 1; }
tail -1 $OUT/pytest_ks.log
timeout -k 10 600 python3 -u bench.py --workload c2 --steps 100 --warmup 20 --no-cpu --no-rocsparse --no-north-star --n-sweep 8,32,128 > $OUT/bench_c2_nsweep.log 2>&1
python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/bench_c2_nsweep.log') if l.startswith('{')][-1]
for x in d['n_sweep']: print(x['N'], x.get('plan'), x.get('kernel'), x.get('kernel_ms'), x.get('hbm_frac'), {k:v.get('kernel_ms') for k,v in x['tried'].items()})"
if [ -n "$DRAM" ]; then
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $OUT/dram_c4o -o p -- python3 bench.py --workload c4o --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/dram_c4o.log 2>&1
python3 scripts/pmc_summary.py $OUT/dram_c4o k_merge_path | tail -4
fi
echo done
