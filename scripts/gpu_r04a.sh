#!/bin/bash
# round 4, first look: k_mfma_ks on C2 -- plan sweep, phase timeline, default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/ks_sweep_c2.py 40,64,80 0,4,8 8,16 > $OUT/sweep.jsonl 2> $OUT/sweep.err
GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so timeout -k 10 120 python3 -u scripts/ks_timeline.py 80 > $OUT/tl80.json 2> $OUT/tl80.err
GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so timeout -k 10 120 python3 -u scripts/mfma_timeline.py 20 > $OUT/tl_rows20.txt 2> $OUT/tl_rows20.err
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json | cut -c1-300
