set -e
mkdir -p gpurun_out/c1
echo '{"WARP_ROWS_GROUPS": 0}' > gpurun_out/c1/nogrp.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/c1/tests.log 2>&1 || { tail -30 gpurun_out/c1/tests.log; exit 1; }
tail -2 gpurun_out/c1/tests.log
timeout -k 10 300 python3 -u scripts/variant_sweep.py c1 f32 8 merge_path:512:1 thread_total:4:1 tblock_warp_total:32:8 tblock_warp_total:64:16 tblock_warp_total:32:32 tblock_warp_total:16:8 tblock_warp_total:64:32 > gpurun_out/c1/sweep.log 2>&1
GS_CONFIG=$PWD/gpurun_out/c1/nogrp.json timeout -k 10 300 python3 -u scripts/variant_sweep.py c1 f32 8 tblock_warp_total:32:8 > gpurun_out/c1/sweep_nogrp.log 2>&1
grep -v amdgpu gpurun_out/c1/sweep.log gpurun_out/c1/sweep_nogrp.log
