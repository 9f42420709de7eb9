# k_merge_path walk attribution (diagnostic, experiments build, wrong results for dbg != 0):
# GS_MP_DEBUG bit 2 gathers B row 0, bit 8 skips the slot scans, bit 16 closes no rows in a round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06zp}; mkdir -p $OUT
export GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so
for wl in c4 c4o; do
  p0=512; st=50; [ $wl = c4o ] && { p0=2048; st=5; }
  for dbg in 0 2 8 16 24 26; do
    GS_MP_DEBUG=$dbg timeout -k 10 300 python3 bench.py --workload $wl --pipeline merge_path --p0 $p0 --steps $st --warmup 3 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/${wl}_d$dbg.log 2>&1 || { echo "$wl $dbg failed"; tail -3 $OUT/${wl}_d$dbg.log; exit 1; }
    python3 -c "
import json
for l in reversed(open('$OUT/${wl}_d$dbg.log').read().strip().splitlines()):
    if l.startswith('{'):
        d=json.loads(l); print('$wl', 'dbg', $dbg, d['ms_per_step']); break
"
  done
done
