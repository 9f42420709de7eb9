"""Kernel time of matrix-core row-block variants per C2 / C5 shape (diagnostic).
usage: shape_sweep.py <shape> [rows:bmw:ksplit[:krot] ...]
shape: c2 (5120^2, 70%) | attn (7168^2, 80%) | fc1 (28672x7168, 80%) | fc2 (7168x28672, 80%)
ksplit 0 = the upload's automatic choice.  Event time over a rotation of >= 600 MB of
the bytes the kernel reads, fp16, N = 32."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import batch as bt  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

shape = sys.argv[1]
N = 32
if shape == "c2":
    M = K = 5120
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
else:
    M, K = bt.C5_SHAPES[shape]
    row, col, val = ds.pruned_weight(M, K, bt.C5_SPARSITY, bt.shape_seed(0, shape))
for spec in sys.argv[2:]:
    r, w, ks, kr = ([int(x) for x in spec.split(":")] + [0])[:4]
    gsa.set_config("MFMA_KSPLIT", ks)
    gsa.set_config("MFMA_KROT", kr)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("tblock_warp_total", N, r, w).compile().upload("f16", 0)
    info = plan.info()
    rd = info["tile_bytes"] or info["device_bytes_A"]
    reps = max(2, int(600e6 // (rd + K * N * 2)) + 1)
    for _ in range(reps - 1):
        plan.add_replica()
    Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
    Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
    plan.spmm_rotate(3 * reps, 0, Bs, Cs)
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.3  # clocks up: ~0.3 s of launches before timing
    while time.perf_counter() < t_end:
        plan.spmm_rotate(reps, 0, Bs, Cs)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(50, 4 * reps)
    e0.record()
    plan.spmm_rotate(n, 0, Bs, Cs)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    alg = len(row) * 4 + (M + 1) * 4 + K * N * 2 + M * N * 2
    print(f"{shape} rows={r} bmw={w} ksplit={ks} krot={kr}: {info.get('device_kernel') or info['kernel_name']} {us:.2f} us, "
          f"{2.0 * len(row) * N / us / 1e3:.0f} GFLOP/s, {alg / us / 1e3:.0f} GB/s "
          f"({alg / us / 1e3 / 8000:.3f} of 8 TB/s)", flush=True)
    plan.free()
    del Bs, Cs
gsa.set_config("MFMA_KSPLIT", 0)
