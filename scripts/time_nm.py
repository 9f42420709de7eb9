"""Time the 2:4 sparse-matrix-core path on C3 (diagnostic; bench.py --workload c3
is the measured line).  usage: time_nm.py [M] [K] [N] [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

a = sys.argv[1:] + [None] * 4
M, K, N, steps = int(a[0] or 28672), int(a[1] or 7168), int(a[2] or 128), int(a[3] or 50)
t0 = time.time()
r, c, v = ds.two_four(M, K, 30)
plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("col_direction_nm", N, 32, 1).compile().upload("f16", 0)
print(f"plan+upload {time.time() - t0:.1f} s", plan.info()["lds_stage"], plan.info()["device_bytes_A"], flush=True)
reps = 3
for _ in range(reps - 1):
    plan.add_replica()
Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
plan.spmm_rotate(5, 0, Bs, Cs)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
plan.spmm_rotate(steps, 0, Bs, Cs)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / steps
nnz = len(r)
byts = nnz * 2 + nnz // 4 + K * N * 2 + M * N * 2
print(f"{M}x{K} N={N}: {ms * 1e3:.1f} us  {2 * nnz * N / ms / 1e9:.1f} TFLOP/s  {byts / ms / 1e6:.1f} GB/s (alg bytes {byts})")
