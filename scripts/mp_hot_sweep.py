"""com-Orkut stand-in (bench.py c4o): merge_path(1024) with the degree renumbering, timed with
several MP_HOT_NT values (gathers of columns >= H non-temporal; read at launch) in interleaved
rounds on one plan (diagnostic A/B).  usage: mp_hot_sweep.py [H,H,...] [rounds] [reps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

hs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,65536,262144,1048576").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
wl = bench.WORKLOADS["c4o"]
M = K = 3072441
N = 8
row, col, val = ds.rmat_torch(M, wl["nnz"], wl["seed"], "cuda", symmetric=True)
plan, Bs, Cs, R, _ = bench.build_plan(gsa, M, K, row, col, val, ("merge_path", 1024, 1), N, "f32", 0, 640.0, 4,
                                      torch.float32, "cuda", torch)
del row, col, val
res = {h: [] for h in hs}
for _ in range(rounds):
    for h in hs:
        gsa.set_config("MP_HOT_NT", h)
        res[h].append(round(bench.event_ms(plan, Bs, Cs, reps, torch), 4))
out = {"plan": "merge_path(1024,1)", "replicas": R, "ms": {str(h): v for h, v in res.items()},
       "median_ms": {str(h): sorted(v)[len(v) // 2] for h, v in res.items()}}
print(json.dumps(out))
