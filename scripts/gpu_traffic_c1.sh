set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tc1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/tc1/fetch -o p -- python3 scripts/variant_sweep.py c1 f32 8 tblock_warp_total:32:8 > gpurun_out/tc1/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/tc1/write -o p -- python3 scripts/variant_sweep.py c1 f32 8 tblock_warp_total:32:8 > gpurun_out/tc1/write.log 2>&1
python3 scripts/traffic_summary.py gpurun_out/tc1 k_warp_rows gpurun_out/tc1/traffic_c1.json 13795144
cat gpurun_out/tc1/traffic_c1.json
