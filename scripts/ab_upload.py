"""A/B of an upload-time config switch on C2 (diagnostic): one plan per value, HIP-event
timing of rotated launches (3 interleaved rounds), C compared with a dense fp32 product.
usage: ab_upload.py KEY v0 v1 [pipeline p0 p1]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

key, vals = sys.argv[1], [int(x) for x in sys.argv[2:4]]
pipe = sys.argv[4] if len(sys.argv) > 4 else "tblock_warp_total"
p0 = int(sys.argv[5]) if len(sys.argv) > 5 else 20
p1 = int(sys.argv[6]) if len(sys.argv) > 6 else 2
M = K = 5120
N = 32
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
plans = []
for v in vals:
    gsa.set_config(key, v)
    pl = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile().upload("f16", 0)
    for _ in range(11):
        pl.add_replica()
    print(key, v, pl.info()["lds_stage"], pl.info()["lds_bytes"], flush=True)
    plans.append(pl)
Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(12)]
Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(12)]
dense = torch.zeros((M, K), device="cuda", dtype=torch.float32)
dense[torch.as_tensor(row.astype("int64")).cuda(), torch.as_tensor(col.astype("int64")).cuda()] = \
    torch.as_tensor(val).half().float().cuda()
full = dense @ Bs[0].float()
for v, pl in zip(vals, plans):
    C = pl.spmm(Bs[0]).float()
    torch.cuda.synchronize()
    err = ((C - full).abs() / full.abs().clamp(min=1.0)).max().item()
    print(key, v, "max rel err vs fp32 dense", err, flush=True)
res = {v: [] for v in vals}
for rnd in range(3):
    for v, pl in zip(vals, plans):
        pl.spmm_rotate(300, 0, Bs, Cs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        pl.spmm_rotate(200, 0, Bs, Cs)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 200 * 1000)
for v in vals:
    print(f"{key}={v}: us/spmm", " ".join(f"{t:.2f}" for t in res[v]))
