"""Kernel time of one (C5-shape, candidate plan) by HIP events over rotated replicas (> 256 MB
of A, past the Infinity Cache); diagnostic for env-selected kernel variants.
usage: shape_time.py <shape> <cand> [sparsity]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import batch as bt  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

N = 32
shape, ci = sys.argv[1], int(sys.argv[2])
sp = float(sys.argv[3]) if len(sys.argv) > 3 else 0.7
m, n = bt.C5_SHAPES[shape]
row, col, val = ds.pruned_weight(m, n, sp, bt.shape_seed(0, shape))
cand = bt.shape_candidates(shape)[ci]
for kv in os.environ.get("SWEEP_CFG", "").split(","):  # KEY=VALUE config overrides
    if kv:
        gsa.set_config(kv.split("=")[0], int(kv.split("=")[1]))
plan = bt.build_plan(gsa, m, n, row, col, val, N, cand, 0)
info = plan.info()
abytes = len(row) * 4
reps = max(2, min(12, int(600e6 // abytes) + 1))
for _ in range(reps - 1):
    plan.add_replica()
Bs = [torch.randn((n, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
Cs = [torch.empty((m, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
plan.spmm_rotate(20, 0, Bs, Cs)
torch.cuda.synchronize()
best = 1e9
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.spmm_rotate(60, 0, Bs, Cs)
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / 60 * 1e3)
print(json.dumps({"shape": shape, "cand": str(cand[:3]), "kernel": info["device_kernel"], "ksplit": info.get("ksplit"),
                  "reps": reps, "us": round(best, 2), "env": {k: v for k, v in os.environ.items() if k.startswith("GS_KS") or k == "SWEEP_CFG"}}),
      flush=True)
plan.free()
