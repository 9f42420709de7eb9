# com-Orkut: merge path with P column partitions (MP_COL_PARTS), one bench line each
OUT=gpurun_out/${TAG:-r06zq}; mkdir -p $OUT
for cfg in "2048 0" "2048 2" "2048 3" "1024 2" "2048 4"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --workload c4o --pipeline merge_path --p0 $1 --config MP_COL_PARTS=$2 --steps 5 --warmup 3 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/c4o_$1_p$2.log 2>&1 || { echo "$cfg failed"; tail -3 $OUT/c4o_$1_p$2.log; exit 1; }
  python3 -c "
import json
for l in reversed(open('$OUT/c4o_$1_p$2.log').read().strip().splitlines()):
    if l.startswith('{'):
        d=json.loads(l); print('merge_path($1) MP_COL_PARTS=$2', d['ms_per_step'], d['roofline']['frac']); break
"
done
