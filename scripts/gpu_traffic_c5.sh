set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tc5
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/tc5/fetch -o p -- python3 bench.py --workload c5 --layers 2 --steps 3 --warmup 1 > gpurun_out/tc5/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/tc5/write -o p -- python3 bench.py --workload c5 --layers 2 --steps 3 --warmup 1 > gpurun_out/tc5/write.log 2>&1
python3 scripts/traffic_c5.py gpurun_out/tc5 2 4 gpurun_out/tc5/traffic_c5.json
