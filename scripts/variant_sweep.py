"""Kernel time of plan variants on one matrix (diagnostic / §8f measurements).
usage: variant_sweep.py <c1|c2|c4> dtype N pipeline:p0:p1 [pipeline:p0:p1 ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

wl, dtype, N = sys.argv[1], sys.argv[2], int(sys.argv[3])
if wl == "c1":
    M, K = 47894, 41550
    row, col, val = ds.random_rows(M, K, 1790490 / 47894, 18)
elif wl == "c2":
    M = K = 5120
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
else:
    M = K = 1000005
    row, col, val = ds.rmat(M, 3105536, 1)
tdt = torch.float16 if dtype == "f16" else torch.float32
e = 2 if dtype == "f16" else 4
for spec in sys.argv[4:]:
    name, p0, p1 = spec.split(":")
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, int(p0), int(p1)).compile().upload(dtype, 0)
    info = plan.info()
    reps = max(2, int(640e6 // (info["device_bytes_A"] + K * N * e)) + 1)
    for _ in range(reps - 1):
        plan.add_replica()
    Bs = [torch.randn((K, N), device="cuda", dtype=tdt) for _ in range(reps)]
    Cs = [torch.empty((M, N), device="cuda", dtype=tdt) for _ in range(reps)]
    plan.spmm_rotate(10, 0, Bs, Cs)
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.3  # clocks up before timing
    while time.perf_counter() < t_end:
        plan.spmm_rotate(reps, 0, Bs, Cs)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.spmm_rotate(100, 0, Bs, Cs)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 100 * 1e3
    print(f"{wl} {dtype} N={N} {name}({p0},{p1}) {info.get('device_kernel') or info['kernel_name']}: {us:.2f} us, "
          f"{2.0 * len(row) * N / us / 1e3:.1f} GFLOP/s, A bytes {info['device_bytes_A']}", flush=True)
    plan.free()
    del Bs, Cs
