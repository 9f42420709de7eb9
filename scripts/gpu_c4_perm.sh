#!/bin/bash
# merge-path column permutation (MP_COL_PERM): parity, C4 webbase on/off, com-Orkut line + traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05c}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py -x -q -k "column_permutation or merge_path" --timeout 120 --timeout-method thread > $OUT/pytest_mp.log 2>&1 || { tail -30 $OUT/pytest_mp.log; exit 1; }
tail -1 $OUT/pytest_mp.log
for pm in 0 1; do
  timeout -k 10 400 python3 -u bench.py --workload c4 --pipeline merge_path --steps 200 --warmup 20 --no-cpu --no-rocsparse --config MP_COL_PERM=$pm > $OUT/bench_c4_perm$pm.log 2>&1
  tail -1 $OUT/bench_c4_perm$pm.log | cut -c1-200
done
timeout -k 10 900 python3 -u bench.py --workload c4o --steps 20 --warmup 5 > $OUT/bench_c4o.log 2>&1
tail -1 $OUT/bench_c4o.log | cut -c1-300
mkdir -p $OUT/tc4o
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/tc4o/$c -o p -- python3 bench.py --workload c4o --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/tc4o/$c.log 2>&1
done
python3 scripts/traffic_summary.py $OUT/tc4o k_merge_path $OUT/traffic_c4o.json 2083887320 || true
python3 scripts/traffic_summary.py $OUT/tc4o k_permute_rows $OUT/traffic_c4o_permute.json || true
echo done
