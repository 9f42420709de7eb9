"""A/B of a launch-time config switch (diagnostic).
usage: ab_config.py KEY v0 v1 [pipeline p0 p1]   (C2)
       WL=c4 ab_config.py MP_WPE 0 6 merge_path 512 1   (C4 stand-in, fp32 N=8)
       WL=c3 ab_config.py NM_NSPLIT 1 2 col_direction_nm 32 1   (C3 2:4, fp16 N=128)
Times 200 rotated SpMMs per setting (HIP events, interleaved settings x3) and checks
every setting's C against the first (bit-exact expected)."""
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
WL = os.environ.get("WL", "c2")
if WL == "c3":
    M, K, N = 28672, 7168, 128
    row, col, val = ds.two_four(M, K, 30)
    dt, tdt = "f16", torch.float16
elif WL == "c4":
    M = K = 1000005
    N = 8
    row, col, val = ds.rmat(M, 3105536, 1, symmetric=False)
    dt, tdt = "f32", torch.float32
else:
    M = K = 5120
    N = 32
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
    dt, tdt = "f16", torch.float16
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile().upload(dt, 0)
reps = 3 if WL == "c3" else 12
for _ in range(reps - 1):
    plan.add_replica()
Bs = [torch.randn((K, N), device="cuda", dtype=tdt) for _ in range(reps)]
Cs = [torch.empty((M, N), device="cuda", dtype=tdt) for _ in range(reps)]
ref = None
for v in vals:
    gsa.set_config(key, v)
    C = plan.spmm(Bs[0])
    torch.cuda.synchronize()
    if ref is None:
        ref = C.clone()
        if WL == "c2":
            dense = torch.zeros((M, K), device="cuda", dtype=torch.float32)
            dense[torch.as_tensor(row.astype("int64")).cuda(), torch.as_tensor(col.astype("int64")).cuda()] = torch.as_tensor(val).float().cuda()
            full = dense @ Bs[0].float()
            print("max abs err vs fp32 dense:", (C.float() - full).abs().max().item())
    else:
        print(key, v, "bit-exact vs first:", torch.equal(C, ref), "max diff", (C.float() - ref.float()).abs().max().item())
res = {v: [] for v in vals}
for rnd in range(3):
    for v in vals:
        gsa.set_config(key, v)
        plan.spmm_rotate(24, 0, Bs, Cs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        plan.spmm_rotate(200, 0, Bs, Cs)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 200 * 1000)
for v in vals:
    print(f"{key}={v}: us/spmm", " ".join(f"{t:.2f}" for t in res[v]))
