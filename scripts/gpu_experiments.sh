#!/bin/bash
# Round-5 A/B experiments on one GPU box (replaces one script per experiment).
# Usage: TAG=r05x bash scripts/gpu_experiments.sh <name> [<name> ...]
#   ks_apart  C2: apart vs overlapped K-split LDS layouts, K splits 2/4/8
#   n128      k_mfma_ks 128-column tiles: parity, C2 dense-width sweep 8/32/128 (+ DRAM=1: com-Orkut
#             TCC_EA0_RDREQ vs TCC_EA0_RDREQ_DRAM)
#   nm4       k_nm_mfma4: 2:4 parity, C3 K-split variants against k_nm_mfma
#   pos8      8-bit K-split positions and 4-wave workgroups: parity, C2 + north_star layer, 20-row S=1
#   c4perm    merge-path column permutation: parity, webbase on/off, com-Orkut line + PMC traffic
#   c4perm2   com-Orkut: gather / scatter / hot-only permutations
#   nm4b      k_nm_mfma4 (half-chunk B ring) against k_nm_mfma on C3
#   exptimeout  the forced K-split timeout test on the experiments library
#   sched     LLVM scheduling strategies (max-ilp / max-memory-clause variant builds) on C2 / C3 / C1
#   nt        A's once-read loads non-temporal (make var VAR_FLAGS=-DGS_A_NT=1): parity, C2/C3/C1/c4o A/B
#   nt2       the same on the north_star layer (c5h) with its per-shape search
#   nt3       KS_NT masks on C2 + the north_star layer, NM_NT over the C3 dense-width sweep
#   nmphase   k_nm_mfma phase stamps + no-B / no-A loop timings on C3 (experiments build)
#   head      KS_HEAD A/B on C2 (KS_NT=1) and the north_star layer
#   c1chunks  k_warp_rows SCF-chunks per slot per pass (WARP_ROWS_CHUNKS) on C1
# Every GPU step runs under its own time limit; the first failure ends the session (set -e).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05x}; mkdir -p $OUT; export TMPDIR=/tmp
set -e
pyt() {  # pytest subset: <log> <files/-k ...>
  local log=$1; shift
  timeout -k 10 600 python3 -u -m pytest "$@" -x -q --timeout 200 --timeout-method thread > $OUT/$log 2>&1 || { tail -30 $OUT/$log; exit 1; }
  tail -1 $OUT/$log
}
line() {  # bench line summary: <log> <label>
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/$1') if l.startswith('{')][-1]
ns=d.get('north_star') or {}
print('$2', d['config'].get('plan'), d['config'].get('kernel'), 'us', round(d['ms_per_step']*1e3,2), 'frac', d['roofline']['frac'],
      'hot_us', round((d['roofline'].get('hot_cache_kernel_ms') or 0)*1e3,2),
      'layer_us', round((ns.get('ms_per_step') or 0)*1e3,1), 'layer_frac', (ns.get('roofline') or {}).get('frac'))"
}
bench() {  # <label> <bench args...>
  local tag=$1; shift
  timeout -k 10 900 python3 -u bench.py "$@" > $OUT/b_$tag.log 2>&1
  line b_$tag.log "$tag"
}
for ex in "$@"; do
  echo "== $ex"
  case $ex in
    ks_apart)
      pyt pytest_apart.log tests/test_gpu_spmm.py -k "overlapped or known_answer_and_c2 or driver_plan"
      c2="--workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --no-north-star --pipeline block_total"
      bench base $c2 --p0 40
      bench ap0_s2 $c2 --p0 40 --config KS_APART=0
      bench ap0_s4 $c2 --p0 40 --config KS_APART=0 --config KS_SPLIT=4
      bench ap1_s4 $c2 --p0 40 --config KS_SPLIT=4
      bench ap0_80s4 $c2 --p0 80 --config KS_APART=0
      bench ap0_80s8 $c2 --p0 80 --config KS_APART=0 --config KS_SPLIT=8 ;;
    n128)
      pyt pytest_ks.log tests/test_gpu_spmm.py -k "mfma_ks or slab or c2"
      bench c2_nsweep --workload c2 --steps 100 --warmup 20 --no-cpu --no-rocsparse --no-north-star --n-sweep 8,32,128
      if [ -n "$DRAM" ]; then
        timeout -s KILL 600 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $OUT/dram_c4o -o p -- \
          python3 bench.py --workload c4o --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/dram_c4o.log 2>&1
      fi ;;
    nm4)
      pyt pytest_nm.log tests/test_gpu_nm.py
      c3="--workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse"
      bench c3_v4auto $c3
      bench c3_v4s1 $c3 --config NM_SPLIT=1
      bench c3_v4s3 $c3 --config NM_SPLIT=3
      bench c3_v4s4 $c3 --config NM_SPLIT=4
      bench c3_classic $c3 --config NM_V4=0 ;;
    nm4b)
      pyt pytest_nm.log tests/test_gpu_nm.py
      c3="--workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse"
      bench c3_classic $c3
      bench c3_v4s2 $c3 --config NM_V4=-1
      bench c3_v4s1 $c3 --config NM_V4=-1 --config NM_SPLIT=1
      bench c3_v4s3 $c3 --config NM_V4=-1 --config NM_SPLIT=3 ;;
    exptimeout)
      GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse_exp.so pyt pytest_exp_timeout.log tests/test_gpu_spmm.py -k "timeout_is_reported" -rA ;;
    pos8)
      pyt pytest_p8.log tests/test_gpu_spmm.py -k "pos8 or mfma_ks or batch or four_waves"
      c2="--workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse"
      bench c2_p80 $c2 --config KS_POS8=0
      bench c2_p81 $c2 --config KS_POS8=1
      bench c2_w4 $c2 --config KS_WAVES=4
      bench c2_w4p8 $c2 --config KS_WAVES=4 --config KS_POS8=1
      bench c2_20s1 $c2 --no-north-star --pipeline block_total --p0 20 --config KS_MIN_ROWS=16
      bench c2_20s1p8 $c2 --no-north-star --pipeline block_total --p0 20 --config KS_MIN_ROWS=16 --config KS_POS8=1 ;;
    c4perm)
      pyt pytest_mp.log tests/test_gpu_spmm.py -k "column_permutation or merge_path"
      c4="--workload c4 --pipeline merge_path --steps 200 --warmup 20 --no-cpu --no-rocsparse"
      bench c4_perm0 $c4 --config MP_COL_PERM=0
      bench c4_perm1 $c4 --config MP_COL_PERM=1
      bench c4o --workload c4o --steps 20 --warmup 5
      mkdir -p $OUT/tc4o
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 600 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/tc4o/$c -o p -- python3 bench.py --workload c4o \
          --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse > $OUT/tc4o/$c.log 2>&1
      done
      python3 scripts/traffic_summary.py $OUT/tc4o k_merge_path $OUT/traffic_c4o.json 2083887320 || true
      python3 scripts/traffic_summary.py $OUT/tc4o k_permute_rows $OUT/traffic_c4o_permute.json || true ;;
    c4perm2)
      pyt pytest_perm.log tests/test_gpu_spmm.py -k "column_permutation"
      c4o="--workload c4o --pipeline merge_path --p0 1024 --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse"
      bench c4o_gather $c4o
      bench c4o_scatter $c4o --config MP_PERM_SCATTER=1
      bench c4o_hot256k $c4o --config MP_PERM_HOT=262144
      bench c4o_hot1m $c4o --config MP_PERM_HOT=1048576 ;;
    nt)  # A's once-read loads non-temporal (libgeneralsparse_var.so built with VAR_FLAGS=-DGS_A_NT=1)
      VAR=$PWD/generalsparse_amd/libgeneralsparse_var.so
      GS_LIBRARY=$VAR pyt pytest_nt.log tests/test_gpu_spmm.py tests/test_gpu_nm.py -k "c2 or mfma_ks or nm or merge_path or headline"
      c2="--workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse"
      bench c2_base $c2
      GS_LIBRARY=$VAR bench c2_nt $c2
      c3="--workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse"
      bench c3_base $c3
      GS_LIBRARY=$VAR bench c3_nt $c3
      c1="--workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse"
      bench c1_base $c1
      GS_LIBRARY=$VAR bench c1_nt $c1
      c4o="--workload c4o --pipeline merge_path --p0 1024 --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse"
      bench c4o_base $c4o
      GS_LIBRARY=$VAR bench c4o_nt $c4o
      GS_LIBRARY=$VAR bench c2_nt2 $c2
      bench c2_base2 $c2 ;;
    nt2)  # the layer and its shapes alone, default vs non-temporal A loads
      VAR=$PWD/generalsparse_amd/libgeneralsparse_var.so
      c5h="--workload c5h --steps 50 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse"
      bench c5h_base $c5h
      GS_LIBRARY=$VAR bench c5h_nt $c5h
      for t in c5h_base c5h_nt; do python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/b_$t.log') if l.startswith('{')][-1]
print('$t', d['ms_per_step'], {k: (v['plan'], v['kernel_us'], {c: x['kernel_us'] for c, x in v['variants'].items()}) for k, v in d['per_shape'].items()})"; done ;;
    nt3)  # KS_NT masks (bit 0 A's groups, bit 1 B's rows) on C2 40-row S=2 and the north_star layer; NM_NT at N = 8 / 32 / 128
      pyt pytest_nt3.log tests/test_gpu_spmm.py tests/test_gpu_nm.py -k "nontemporal or driver_plan or headline"
      c2="--workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --pipeline block_total --p0 40"
      for x in 0 1 2 3 0 1 2 3; do bench c2_nt$x $c2 --config KS_NT=$x; done
      c3="--workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse --pipeline col_direction_nm --n-sweep 8,32,128"
      for x in 0 1; do
        bench c3_nmnt$x $c3 --config NM_NT=$x
        python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/b_c3_nmnt$x.log') if l.startswith('{')][-1]
print('c3 NM_NT=$x sweep', [(r['N'], r.get('kernel_ms')) for r in d.get('n_sweep', [])])"
      done ;;
    nmphase)  # k_nm_mfma phase stamps and the loop without B / A loads (experiments build)
      EXP=$PWD/generalsparse_amd/libgeneralsparse_exp.so
      for dbg in 0 1 2 8; do GS_LIBRARY=$EXP GS_NM_DEBUG=$dbg timeout -k 10 300 python3 -u scripts/nm_phases.py 128 50; done
      GS_LIBRARY=$EXP GS_NM_DEBUG=4 timeout -k 10 300 python3 -u scripts/nm_phases.py 128 > $OUT/nm_stamps.txt 2>&1
      grep "wave" $OUT/nm_stamps.txt | head -30 ;;
    head)  # KS_HEAD (head steps at fixed slots) on C2 40-row (with KS_NT=1) + the north_star layer
      pyt pytest_head.log tests/test_gpu_spmm.py -k "head_steps or nontemporal or driver_plan or headline or mfma_ks_matches"
      c2="--workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --pipeline block_total --p0 40 --config KS_NT=1"
      for x in 0 1 0 1; do bench c2_head$x $c2 --config KS_HEAD=$x; done ;;
    c1chunks)  # k_warp_rows chunks per slot per pass on C1 (and the C2 / C4 gather candidates' parity)
      pyt pytest_chunks.log tests/test_gpu_spmm.py -k "warp_rows_chunks or PIPES or pipes"
      c1="--workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 32 --p1 8"
      for x in 1 2 3 1 2 3; do bench c1_ch$x $c1 --config WARP_ROWS_CHUNKS=$x; done
      bench c1_auto --workload c1 --steps 200 --warmup 20 --no-cpu ;;
    n128b)  # C2 at N = 128: row-block height x K split on k_mfma_ks (CT = 8 up to 48 rows)
      for p0 in 32 40 48; do for sp in 0 3 4; do
        timeout -k 10 600 python3 -u bench.py --workload c2 --steps 20 --warmup 5 --no-cpu --no-rocsparse --no-north-star \
          --pipeline block_total --p0 $p0 --n-sweep 128 --config KS_SPLIT=$sp > $OUT/n128_${p0}_$sp.log 2>&1
        python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/n128_${p0}_$sp.log') if l.startswith('{')][-1]
print('rows $p0 split $sp', [(r['N'], r.get('kernel'), r.get('kernel_ms'), r.get('hbm_frac')) for r in d['n_sweep']])"
      done; done ;;
    n128nt)  # C2 at N = 128 with KS_NT on the 128-column tiles: parity, then the dense-width sweep (candidates incl. KS_NT)
      pyt pytest_n128nt.log tests/test_gpu_spmm.py -k "nontemporal"
      bench c2_nsweep --workload c2 --steps 20 --warmup 5 --no-cpu --no-rocsparse --no-north-star --n-sweep 8,32,128
      python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/b_c2_nsweep.log') if l.startswith('{')][-1]
for r in d['n_sweep']: print(r['N'], r.get('plan'), r.get('kernel_ms'), r.get('hbm_frac'), {k: v.get('kernel_ms') for k, v in r['tried'].items()})" ;;
    graph)  # C2 launches in a HIP graph vs one by one
      for x in "40 200 KS_NT=1" "40 200 KS_NT=0" "80 200 KS_NT=1"; do timeout -k 10 300 python3 -u scripts/graph_probe.py $x; done ;;
    wrows)  # k_warp_rows / k_warp_rows_mc after the split: parity, C1 line, C2 gather candidates
      pyt pytest_wrows.log tests/test_gpu_spmm.py -k "warp_rows or PIPES or pipes or tblock or mfma_ks or nontemporal or head"
      bench c1 --workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse
      bench c2 --workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --no-north-star --n-sweep 128
      python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/b_c2.log') if l.startswith('{')][-1]
print({k: v.get('kernel_ms') for k, v in d['variants'].items()})
print('N=128', [(r.get('plan'), r.get('kernel_ms'), r.get('hbm_frac'), {k: v.get('kernel_ms') for k, v in r['tried'].items()}) for r in d['n_sweep']])" ;;
    prio)  # KS_PRIO re-check on the round-5 kernel (head steps, KS_NT) : C2 + the north_star layer
      c2="--workload c2 --steps 200 --warmup 50 --no-cpu --no-rocsparse --pipeline block_total --p0 40 --config KS_NT=1"
      for x in 1 0 2 1 0 2; do bench c2_prio$x $c2 --config KS_PRIO=$x; done ;;
    krot)  # C3 k_nm_mfma: every workgroup from its own B chunk (MFMA_KROT=1) vs all from chunk 0
      pyt pytest_krot.log tests/test_gpu_nm.py -k "c3_scale or linearity"
      c3="--workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse --pipeline col_direction_nm"
      for x in 0 1 0 1; do bench c3_krot$x $c3 --config MFMA_KROT=$x; done ;;
    c1plans)  # C1: tblock_warp_total(rows per BMTB, rows per BMW) sweep on k_warp_rows_mc
      for pp in ${C1PLANS:-16_8 32_8 64_8 128_8 32_16 64_16 32_4 64_32}; do
        set -- ${pp/_/ }
        bench c1_$1_$2 --workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 $1 --p1 $2
      done ;;
    c4plans)  # C4 webbase: other plans beside the merge path
      for pp in "tblock_warp_total 32 8" "tblock_warp_total 64 16" "tblock_warp_total 128 32" "merge_path 128 1" "merge_path 256 1" "balanced_warp_total 64 1" "balanced_warp_total 256 1"; do
        set -- $pp
        bench c4_$1_$2_$3 --workload c4 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline $1 --p0 $2 --p1 $3 || true
      done ;;
    c2rows)  # C2 k_mfma_ks row-block height x K split with KS_NT=1 and head steps
      c2="--workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --no-north-star --pipeline block_total --config KS_NT=1"
      for pp in "32 0" "40 0" "48 0" "56 0" "64 0" "80 0" "48 2" "56 2" "64 2" "40 3"; do
        set -- $pp
        bench c2_$1_$2 $c2 --p0 $1 --config KS_SPLIT=$2 --config KS_MIN_ROWS=32 || true
      done ;;
    c5grp)  # C5 batch: launches per matrix over two streams (default) vs grouped k_mfma_ks launches
      bench c5_streams --workload c5 --steps 20 --warmup 10 --no-cpu --no-rocsparse
      bench c5_group --workload c5 --steps 20 --warmup 10 --no-cpu --no-rocsparse --group 1 --streams 1
      bench c5_group2 --workload c5 --steps 20 --warmup 10 --no-cpu --no-rocsparse --group 1 --streams 2 ;;
    c4owork)  # com-Orkut merge-path work size
      for ws in 2048 4096; do
        bench c4o_$ws --workload c4o --pipeline merge_path --p0 $ws --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse || true
      done ;;
    sched)  # LLVM scheduling strategies for the device code: libgeneralsparse_var_ilp.so
      # (VAR_FLAGS="-mllvm -amdgpu-sched-strategy=max-ilp") and _mclause.so (max-memory-clause)
      ILP=$PWD/generalsparse_amd/libgeneralsparse_var_ilp.so
      MCL=$PWD/generalsparse_amd/libgeneralsparse_var_mclause.so
      GS_LIBRARY=$ILP pyt pytest_ilp.log tests/test_gpu_spmm.py tests/test_gpu_nm.py -k "driver_plan or nontemporal or head_steps or nm_matches"
      GS_LIBRARY=$MCL pyt pytest_mcl.log tests/test_gpu_spmm.py tests/test_gpu_nm.py -k "driver_plan or nontemporal or head_steps or nm_matches"
      c2="--workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --no-north-star --pipeline block_total --p0 40 --config KS_NT=1"
      c3="--workload c3 --steps 100 --warmup 20 --no-cpu --no-rocsparse"
      c1="--workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse"
      for r in 1 2; do
        bench c2_base$r $c2; GS_LIBRARY=$ILP bench c2_ilp$r $c2; GS_LIBRARY=$MCL bench c2_mcl$r $c2
      done
      bench c3_base $c3; GS_LIBRARY=$ILP bench c3_ilp $c3; GS_LIBRARY=$MCL bench c3_mcl $c3
      bench c1_base $c1; GS_LIBRARY=$ILP bench c1_ilp $c1; GS_LIBRARY=$MCL bench c1_mcl $c1 ;;
    sched2)  # max-ilp repeat: C2 x4, C1 x2, the north_star layer (c5h) x1, alternating
      ILP=$PWD/generalsparse_amd/libgeneralsparse_var_ilp.so
      c2="--workload c2 --steps 200 --warmup 20 --no-cpu --no-rocsparse --no-north-star --pipeline block_total --p0 40 --config KS_NT=1"
      c1="--workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 64 --p1 16"
      c5h="--workload c5h --steps 100 --warmup 10 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse"
      for r in 1 2 3 4; do bench c2_base$r $c2; GS_LIBRARY=$ILP bench c2_ilp$r $c2; done
      for r in 1 2; do bench c1_base$r $c1; GS_LIBRARY=$ILP bench c1_ilp$r $c1; done
      bench c5h_base $c5h; GS_LIBRARY=$ILP bench c5h_ilp $c5h ;;
    sched3)  # max-ilp on the gather kernels: C4 webbase (k_merge_path) x2, com-Orkut x1, C1 x1
      ILP=$PWD/generalsparse_amd/libgeneralsparse_var_ilp.so
      c4="--workload c4 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline merge_path --p0 256"
      c4o="--workload c4o --pipeline merge_path --p0 2048 --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse"
      c1="--workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 64 --p1 16"
      for r in 1 2; do bench c4_base$r $c4; GS_LIBRARY=$ILP bench c4_ilp$r $c4; done
      bench c4o_base $c4o; GS_LIBRARY=$ILP bench c4o_ilp $c4o
      GS_LIBRARY=$ILP bench c1_ilp3 $c1; bench c1_base3 $c1 ;;
    c1ilp)  # C1 under the max-ilp gather build: chunks per pass x plan
      for pp in "64 16 3" "64 16 2" "64 16 1" "32 16 3" "48 16 3" "64 8 3" "64 16 3" "32 8 2"; do
        set -- $pp
        bench c1_$1_$2_ch$3 --workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 $1 --p1 $2 --config WARP_ROWS_CHUNKS=$3 || true
      done ;;
    c1mc5)  # k_warp_rows_mc with 5-chunk capacity at 3 waves per SIMD (libgeneralsparse_var.so built with
      # VAR_FLAGS="-DGS_WR_MAXCH=5 -DGS_WR_WPE=3") against the default (3 chunks, 4 waves)
      VAR=$PWD/generalsparse_amd/libgeneralsparse_var.so
      GS_LIBRARY=$VAR pyt pytest_mc5.log tests/test_gpu_spmm.py -k "warp_rows_chunks or spmm_matches_oracle"
      c1="--workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 64 --p1 16"
      bench c1_def $c1
      for x in 3 4 5; do GS_LIBRARY=$VAR bench c1_mc5_ch$x $c1 --config WARP_ROWS_CHUNKS=$x; done
      GS_LIBRARY=$VAR bench c1_mc5_128_32_ch5 --workload c1 --steps 200 --warmup 20 --no-cpu --no-rocsparse --pipeline tblock_warp_total --p0 128 --p1 32 --config WARP_ROWS_CHUNKS=5
      bench c1_def2 $c1 ;;
    *) echo "unknown experiment $ex"; exit 2 ;;
  esac
done
echo "session $TAG done"
