# k_lds_rows_rs (fp32 C2, one row per slot): parity tests, then a plan A/B (scripts/ab_plans.py WL=c2f)
mkdir -p gpurun_out/${TAG:-r06y}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_spmm.py -x -q --timeout 120 --timeout-method thread -k "rowslot or dma_fp32" > gpurun_out/${TAG:-r06y}/test_rs.log 2>&1 || { tail -30 gpurun_out/${TAG:-r06y}/test_rs.log; exit 1; }
tail -2 gpurun_out/${TAG:-r06y}/test_rs.log
WL=c2f timeout -k 10 400 python3 -u scripts/ab_plans.py "$@" > gpurun_out/${TAG:-r06y}/ab_rs.txt 2>&1
python3 -c "
import json
for l in open('gpurun_out/${TAG:-r06y}/ab_rs.txt'):
    if 'variant' in l:
        d=json.loads(l); print(d['variant'], d['kernel'], d['median_us'], d['ksplit'])
"
