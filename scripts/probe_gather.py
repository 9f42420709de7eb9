"""Probe what bounds the row-wave kernel on C2-shaped inputs (diagnostic only).

Variants keep the per-row nnz pattern and change B's footprint / row width:
  c2        5120x5120 70% pruned, fp16, N=32 (64-B B rows, B = 320 KB)
  c2_l1     same rows, cols folded mod 256 (B = 16 KB: fits L1)
  c2_n64    N=64 (128-B B rows)
  c2_n16    N=16 (32-B B rows)
  c2_f32    fp32, N=32 (128-B rows)
Prints kernel ms (events over rotated replicas) per variant."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402


def timeit(M, K, row, col, val, N, dtype, pipeline="tblock_warp_total", p0=4, reps=8, steps=100):
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipeline, N, p0, 1).compile().upload(dtype, 0)
    for _ in range(reps - 1):
        plan.add_replica()
    tdt = torch.float16 if dtype == "f16" else torch.float32
    Bs = [torch.randn((K, N), device="cuda", dtype=tdt) for _ in range(reps)]
    Cs = [torch.empty((M, N), device="cuda", dtype=tdt) for _ in range(reps)]
    plan.spmm_rotate(20, 0, Bs, Cs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.spmm_rotate(steps, 0, Bs, Cs)
    e1.record()
    torch.cuda.synchronize()
    plan.free()
    return e0.elapsed_time(e1) / steps


def main():
    M = K = 5120
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
    out = {}
    out["c2"] = timeit(M, K, row, col, val, 32, "f16")
    # fold columns into 256 distinct B rows, keep rows sorted/unique per row
    c2 = (col % 256)
    key = row.astype(np.int64) * 256 + c2.astype(np.int64)
    key = np.unique(key)
    r2, cc2 = (key // 256).astype(np.uint64), (key % 256).astype(np.uint64)
    out["c2_l1_fold256"] = timeit(M, 256, r2, cc2, np.ones(len(r2), np.float32), 32, "f16")
    out["c2_l1_nnz"] = int(len(r2))
    out["c2_n64"] = timeit(M, K, row, col, val, 64, "f16")
    out["c2_n16"] = timeit(M, K, row, col, val, 16, "f16")
    out["c2_f32_n32"] = timeit(M, K, row, col, val, 32, "f32")
    out["c2_block_total"] = timeit(M, K, row, col, val, 32, "f16", "block_total", 0)
    out["c2_tblock16"] = timeit(M, K, row, col, val, 32, "f16", "tblock_warp_total", 16)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
