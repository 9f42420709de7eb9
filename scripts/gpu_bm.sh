#!/bin/bash
# C2 k_mfma_rows attribution: diagnostic builds without parts of the work (GS_MFMA_DEBUG bits)
mkdir -p gpurun_out
for d in 0 1 2 4 10 11 15; do
  GS_MFMA_DEBUG=$d timeout -k 10 120 python bench.py --pipeline tblock_warp_total --p0 20 --p1 2 --steps 200 --warmup 200 --no-cpu --no-rocsparse > gpurun_out/md$d.log 2>&1 || break
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/md$d.log') if l.startswith('{')][-1]
print('dbg $d', d['roofline']['kernel_ms'], d['roofline']['hot_cache_kernel_ms'])"
done
