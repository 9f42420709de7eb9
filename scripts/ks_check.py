"""k_mfma_ks check + timing (diagnostic): parity vs a dense fp32 torch product on small
ragged shapes and on C2, then event time of C2 plans with rotated replicas.
usage: ks_check.py [plans...]   plan = pipeline:p0:p1[:KEY=V,...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402


def dense_ref(M, K, row, col, val, B):
    A = torch.zeros((M, K), dtype=torch.float32, device="cuda")
    A.index_put_((torch.as_tensor(row.astype(np.int64)).cuda(), torch.as_tensor(col.astype(np.int64)).cuda()),
                 torch.as_tensor(val.astype(np.float16).astype(np.float32)).cuda(), accumulate=True)
    return A @ B.float()


def check(M, K, N, row, col, val, pipe, p0, p1, cfg=()):
    for k, v in cfg:
        gsa.set_config(k, v)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile().upload("f16", 0)
    info = plan.info()
    B = torch.empty((K, N), device="cuda", dtype=torch.float16).uniform_(-1, 1)
    C = plan.spmm(B)
    C2 = plan.spmm(B)
    torch.cuda.synchronize()
    ref = dense_ref(M, K, row, col, val, B)
    err = ((C.float() - ref).abs() / (1 + ref.abs())).max().item()
    det = torch.equal(C, C2)
    print(f"M={M} K={K} N={N} {pipe}({p0},{p1}) {dict(cfg)} kernel={info.get('device_kernel')} "
          f"rel_err={err:.3g} deterministic={det}", flush=True)
    plan.free()
    for k, v in cfg:
        gsa.set_config(k, {"MFMA_KS": 1, "KS_SPLIT": 0, "KS_MIN_ROWS": 40}.get(k, v))
    return err < 0.1 and det


def timeit(M, K, N, row, col, val, pipe, p0, p1, cfg=(), reps=200):
    for k, v in cfg:
        gsa.set_config(k, v)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile().upload("f16", 0)
    info = plan.info()
    nrep = max(2, int(640e6 // (info["tile_bytes"] or info["device_bytes_A"])) + 1)
    for _ in range(nrep - 1):
        plan.add_replica()
    Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(nrep)]
    Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(nrep)]
    plan.spmm_rotate(50, 0, Bs, Cs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.spmm_rotate(reps, 0, Bs, Cs)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    nnz = len(row)
    alg = nnz * 4 + (M + 1) * 4 + K * N * 2 + M * N * 2
    print(f"TIME {pipe}({p0},{p1}) {dict(cfg)} {info.get('device_kernel')} ksplit={info.get('ksplit')} "
          f"{us:.2f} us  {2 * nnz * N / us / 1e3:.0f} GFLOP/s  frac={alg / us / 1e3 / 8000:.3f}", flush=True)
    plan.free()
    del Bs, Cs
    torch.cuda.empty_cache()
    for k, v in cfg:
        gsa.set_config(k, {"MFMA_KS": 1, "KS_SPLIT": 0, "KS_MIN_ROWS": 40}.get(k, v))


def main():
    ok = True
    rng_cases = [(300, 1000, 0.3, 48), (257, 4099, 0.25, 80), (1000, 777, 0.5, 64), (96, 96, 0.9, 48)]
    for (M, K, dens, rb) in rng_cases:
        row, col, val = ds.random_rows(M, K, dens * K, seed=M + K, empty_frac=0.05)
        for N in (16, 32, 64):
            ok &= check(M, K, N, row, col, val, "block_total", rb, 1)
    row, col, val = ds.pruned_weight(5120, 5120, 0.7, 13)
    for cfg in ((), (("KS_SPLIT", 2),), (("KS_SPLIT", 8),)):
        ok &= check(5120, 5120, 32, row, col, val, "block_total", 80, 1, cfg)
    print("PARITY", "OK" if ok else "FAIL", flush=True)
    for (pipe, p0, p1, cfg) in [("tblock_warp_total", 20, 2, ()), ("block_total", 80, 1, ()),
                                ("block_total", 80, 1, (("KS_SPLIT", 8),)), ("block_total", 64, 1, ()),
                                ("block_total", 48, 1, ()), ("tblock_warp_total", 80, 2, ())]:
        timeit(5120, 5120, 32, row, col, val, pipe, p0, p1, cfg)


if __name__ == "__main__":
    main()
