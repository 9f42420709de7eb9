#!/bin/bash
# Round-4 final-tree session.  PART=a: the -m gpu suite + smoke; PART=b: bench lines + a
# rocprofv3 --kernel-trace --stats run of the same command per workload ($WLS); PART=c: PMC
# traffic passes (C5 batch, headline-layer candidates, com-Orkut stand-in).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04z}
mkdir -p $OUT
export TMPDIR=/tmp
set -e
if [ "$PART" = "a" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -7 $OUT/smoke.log
fi
if [ "$PART" = "b" ]; then
  for wl in $WLS; do
    steps=200; psteps=100; extra=""
    if [ "$wl" = "c5" ]; then steps=20; psteps=5; fi
    if [ "$wl" = "c5h" ]; then steps=50; psteps=10; fi
    if [ "$wl" = "c4o" ]; then steps=20; psteps=5; fi
    timeout -k 10 900 python3 -u bench.py --workload $wl --steps $steps --warmup 20 > $OUT/bench_$wl.log 2>&1
    tail -1 $OUT/bench_$wl.log | cut -c1-240
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o p -- python3 bench.py --workload $wl --steps $psteps --warmup 10 --no-cpu --no-rocsparse > $OUT/prof_$wl.log 2>&1
    echo "prof $wl done"
  done
fi
if [ "$PART" = "c" ] || [ "$PART" = "c5t" ]; then
  mkdir -p $OUT/tc5
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/tc5/fetch -o p -- python3 bench.py --workload c5 --layers 2 --steps 3 --warmup 1 --no-cpu > $OUT/tc5/fetch.log 2>&1
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/tc5/write -o p -- python3 bench.py --workload c5 --layers 2 --steps 3 --warmup 1 --no-cpu > $OUT/tc5/write.log 2>&1
  python3 scripts/traffic_c5.py $OUT/tc5 2 4 $OUT/traffic_c5.json
fi
if [ "$PART" = "c" ] || [ "$PART" = "c5ht" ]; then
  rm -rf $OUT/tc5h; mkdir -p $OUT/tc5h
  for sc in $(python3 scripts/traffic_c5h.py list); do
    s=${sc%%:*}; c=${sc##*:}
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/tc5h/fetch_${s}_${c} -o p -- python3 scripts/traffic_c5h.py run $s $c 8 > $OUT/tc5h/fetch_${s}_${c}.log 2>&1
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/tc5h/write_${s}_${c} -o p -- python3 scripts/traffic_c5h.py run $s $c 8 > $OUT/tc5h/write_${s}_${c}.log 2>&1
    echo "tc5h $s $c"
  done
  python3 scripts/traffic_c5h.py summarize $OUT/tc5h 8 $OUT/traffic_c5h.json > /dev/null
fi
if [ "$PART" = "c" ] || [ "$PART" = "c4ot" ]; then
  mkdir -p $OUT/tc4o
  timeout -s KILL 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/tc4o/fetch -o p -- python3 bench.py --workload c4o --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/tc4o/fetch.log 2>&1
  timeout -s KILL 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/tc4o/write -o p -- python3 bench.py --workload c4o --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/tc4o/write.log 2>&1
  python3 scripts/traffic_summary.py $OUT/tc4o k_merge_path $OUT/traffic_c4o.json 2083887320 || true
  echo "traffic done"
fi
