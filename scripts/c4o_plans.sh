# com-Orkut stand-in: one bench line per plan (merge path against the balanced / row-per-wave families)
mkdir -p gpurun_out/${TAG:-r06zg}
for pl in "balanced_warp_total 512" "balanced_warp_total 2048" "balanced_block_total 2048" "merge_path 2048"; do
  set -- $pl
  timeout -k 10 300 python3 -u bench.py --workload c4o --pipeline $1 --p0 $2 --steps 5 --warmup 2 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > gpurun_out/${TAG:-r06zg}/c4o_$1_$2.json 2> gpurun_out/${TAG:-r06zg}/c4o_$1_$2.err || { echo "$pl failed"; tail -5 gpurun_out/${TAG:-r06zg}/c4o_$1_$2.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${TAG:-r06zg}/c4o_$1_$2.json').read().strip().splitlines()[-1])
print('$pl', d['config']['kernel'], d['ms_per_step'], d['roofline']['frac'])
"
done
