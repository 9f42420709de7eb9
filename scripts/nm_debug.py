import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import generalsparse_amd as gsa, oracle_ffi as ofi
from generalsparse_amd import datasets as ds
for N in (32, 64, 128):
  for M, K in ((96, 512), (300, 1024)):
    r, c, v = ds.two_four(M, K, 30 + M)
    plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("col_direction_nm", N, 32, 1).compile().upload("f16", 0)
    B = np.random.default_rng(M + K).uniform(-1, 1, (K, N)).astype(np.float16)
    ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    C = plan.spmm(torch.from_numpy(B).cuda()).float().cpu().numpy()
    err = np.abs(C - ref) / np.maximum(1, np.abs(ref))
    bad = np.argwhere(err > 0.1)
    print(N, M, K, plan.info()["device_kernel"], plan.info()["ksplit"], "bad", len(bad), "rows", sorted(set(bad[:, 0].tolist()))[:20], "cols", sorted(set(bad[:, 1].tolist()))[:40])
    if len(bad):
        i, j = bad[0]; print("  C", C[i, j], "ref", ref[i, j])
