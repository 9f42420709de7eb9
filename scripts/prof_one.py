"""Run one C2 plan for `steps` rotated launches (profiling target; diagnostic only).
usage: prof_one.py [pipeline] [p0] [p1] [dtype] [N] [steps] [KEY=VALUE ...] (config overrides, e.g. KS_NT=1)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

over = [x for x in sys.argv[1:] if "=" in x]
for kv in over:
    k, v = kv.split("=", 1)
    gsa.set_config(k, int(v))
a = [x for x in sys.argv[1:] if "=" not in x] + [None] * 6
pipe = a[0] or "tblock_warp_total"
p0, p1 = int(a[1] or 20), int(a[2] or 2)
dtype, N, steps = a[3] or "f16", int(a[4] or 32), int(a[5] or 200)
M = K = 5120
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile().upload(dtype, 0)
reps = 8
for _ in range(reps - 1):
    plan.add_replica()
tdt = torch.float16 if dtype == "f16" else torch.float32
Bs = [torch.randn((K, N), device="cuda", dtype=tdt) for _ in range(reps)]
Cs = [torch.empty((M, N), device="cuda", dtype=tdt) for _ in range(reps)]
plan.spmm_rotate(steps, 0, Bs, Cs)
torch.cuda.synchronize()
print(plan.info())
