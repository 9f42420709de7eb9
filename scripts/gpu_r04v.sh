#!/bin/bash
# PMC traffic passes on the final tree's chosen plans: C2 block_total(40,1) (k_mfma_ks), com-Orkut
# merge_path(1024), the C5 batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04v
mkdir -p $OUT/c2 $OUT/c4o
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/c2/$c -o p -- python3 bench.py --steps 50 --warmup 5 --pipeline block_total --p0 40 --p1 1 --no-cpu --no-rocsparse > $OUT/c2/$c.log 2>&1
done
python3 scripts/traffic_summary.py $OUT/c2 k_mfma_ks $OUT/traffic_c2.json 32133124
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/c4o/$c -o p -- python3 bench.py --workload c4o --pipeline merge_path --p0 1024 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/c4o/$c.log 2>&1
done
python3 scripts/traffic_summary.py $OUT/c4o k_merge_path $OUT/traffic_c4o.json 2083887320 || true
TAG=r04v PART=c5t bash scripts/gpu_r04z.sh
cat $OUT/traffic_c2.json; echo; cat $OUT/traffic_c4o.json; echo; head -c 600 $OUT/traffic_c5.json
