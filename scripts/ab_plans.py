"""A/B of upload-time plan variants (diagnostic): each variant is built and uploaded with its own
config overrides, then all are timed interleaved (ROUNDS rounds x 200 rotated SpMMs, HIP events)
and every C is compared with the first variant's (bit-exact expected for deterministic kernels).
usage: WL=c3 ab_plans.py '["col_direction_nm",32,1,{"NM_TILES":7}]' '["col_direction_nm",32,1,{"NM_TILES":8}]'
WL: c2 (5120^2 70% fp16 N=32), c3 (28672x7168 2:4 fp16 N=128), c4 (webbase stand-in fp32 N=8),
c2f (C2 at fp32); N overrides the dense width.  Prints one JSON line per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

WL = os.environ.get("WL", "c2")
ROUNDS = int(os.environ.get("ROUNDS", "5"))
if WL == "c3":
    M, K, N = 28672, 7168, 128
    row, col, val = ds.two_four(M, K, 30)
    dt, tdt = "f16", torch.float16
elif WL == "c4":
    M = K = 1000005
    N = 8
    row, col, val = ds.rmat(M, 3105536, 1, symmetric=False)
    dt, tdt = "f32", torch.float32
elif WL == "pw":  # any pruned-weight shape: M, K, SP (sparsity), DT (f16 / f32)
    M, K, N = int(os.environ["M"]), int(os.environ["K"]), 32
    row, col, val = ds.pruned_weight(M, K, float(os.environ.get("SP", "0.7")), 13)
    dt = os.environ.get("DT", "f16")
    tdt = torch.float16 if dt == "f16" else torch.float32
else:
    M = K = 5120
    N = 32
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
    dt, tdt = ("f32", torch.float32) if WL == "c2f" else ("f16", torch.float16)
N = int(os.environ.get("N", N))
variants = [json.loads(a) for a in sys.argv[1:]]
plans = []
for v in variants:
    name, p0, p1 = v[:3]
    over = v[3] if len(v) > 3 else {}
    old = {k: gsa.get_config(k) for k in over}
    try:
        for k, x in over.items():
            gsa.set_config(k, x)
        p = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile().upload(dt, 0)
    finally:
        for k, x in old.items():
            gsa.set_config(k, x)
    # rotated copies: >= 1 GB and >= 4 copies, so every launch reads A past the 256 MB Infinity Cache
    reps = max(4, int(1e9 // (p.info()["device_bytes_A"] + K * N * (2 if dt == "f16" else 4))))
    for _ in range(reps - 1):
        p.add_replica()
    plans.append((v, p, reps))
R = max(r for _, _, r in plans)
Bs = [torch.randn((K, N), device="cuda", dtype=tdt) for _ in range(R)]
Cs = [torch.empty((M, N), device="cuda", dtype=tdt) for _ in range(R)]
ref = None
same, rel = [], []
for v, p, r in plans:
    C = p.spmm(Bs[0])
    torch.cuda.synchronize()
    if ref is None:
        ref = C.clone()
    same.append(bool(torch.equal(C, ref)))
    rel.append(((C.float() - ref.float()).abs() / ref.float().abs().clamp(min=1.0)).max().item())
res = [[] for _ in plans]
for rnd in range(ROUNDS):
    for i, (v, p, r) in enumerate(plans):
        rot = p.rotation(Bs[:r], Cs[:r])
        rot.run(24, 0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        rot.run(200, 0)
        e1.record()
        torch.cuda.synchronize()
        res[i].append(e0.elapsed_time(e1) / 200 * 1000)
for i, (v, p, r) in enumerate(plans):
    info = p.info()
    print(json.dumps({"variant": v, "kernel": info["device_kernel"], "us": [round(t, 2) for t in res[i]],
                      "median_us": round(sorted(res[i])[len(res[i]) // 2], 2), "bit_identical_to_first": same[i], "max_rel_diff_to_first": rel[i],
                      "replicas": r, "nm_tiles": info.get("nm_tiles"), "ksplit": info.get("ksplit")}))
