# Parameters of scripts/gpu_session.sh per workload (sourced).
# bench_steps / prof_steps: timed steps of the bench line and of its rocprofv3 run;
# pmc_cmd: the program a PMC pass profiles (the bench's chosen plan alone, bounded launches).
bench_steps() { case $1 in c5|c4o) echo 20 ;; c5h) echo 50 ;; *) echo 200 ;; esac; }
prof_steps() { case $1 in c5|c4o) echo 5 ;; c5h) echo 10 ;; *) echo 100 ;; esac; }
pmc_cmd() {
  case $1 in
    c2) echo "python3 scripts/prof_one.py block_total 40 1 f16 32 100 ${C2_PMC_CONFIG:-KS_NT=1}" ;;
    c3) echo "python3 bench.py --workload c3 --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse" ;;
    c4o) echo "python3 bench.py --workload c4o --pipeline merge_path --p0 512 --steps 3 --warmup 1 --search-reps 2 --search-rounds 1 --no-cpu --no-rocsparse" ;;
    c5h) echo "python3 bench.py --workload c5h --steps 5 --warmup 2 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse" ;;
    *) echo "python3 bench.py --workload $1 --steps 20 --warmup 5 --search-reps 5 --search-rounds 1 --no-cpu --no-rocsparse" ;;
  esac
}
