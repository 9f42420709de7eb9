"""Time C2 (5120x5120, 70% pruned, N=32) under several tblock_warp_total
shapes with and without the LDS-staged kernel (diagnostic only)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402


def timeit(M, K, row, col, val, N, dtype, p0, p1, reps=8, steps=100, pipe="tblock_warp_total"):
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile()
    plan.upload(dtype, 0)
    for _ in range(reps - 1):
        plan.add_replica()
    info = plan.info()
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
    return {"ms": round(e0.elapsed_time(e1) / steps, 5), "lds": info["lds_stage"], "KC": info["lds_kc"],
            "chunks": info["lds_chunks"], "waves": info["lds_waves"], "lds_bytes": info["lds_bytes"]}


def main():
    M = K = 5120
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
    out = {}
    for p0 in (20, 16, 32, 10, 40, 64):
        k = f"mfma_block_total_{p0}"
        out[k] = timeit(M, K, row, col, val, 32, "f16", p0, 1, pipe="block_total")
        print(json.dumps({k: out[k]}), flush=True)
    for n in (16, 64, 128):
        k = f"mfma_block_total_20_n{n}"
        out[k] = timeit(M, K, row, col, val, n, "f16", 20, 1, pipe="block_total")
        print(json.dumps({k: out[k]}), flush=True)
    gsa.set_config("MFMA_TILES", 0)
    shapes = [(20, 2), (24, 2)]
    for p0, p1 in shapes:
        out[f"f16_{p0}x{p1}"] = timeit(M, K, row, col, val, 32, "f16", p0, p1)
        print(json.dumps({f"f16_{p0}x{p1}": out[f"f16_{p0}x{p1}"]}), flush=True)
    out["f32_20x2"] = timeit(M, K, row, col, val, 32, "f32", 20, 2)
    out["f16_n64_20x2"] = timeit(M, K, row, col, val, 64, "f16", 20, 2)
    out["f16_n16_20x2"] = timeit(M, K, row, col, val, 16, "f16", 20, 2)
    gsa.set_config("LDS_STAGE_B", 0)
    out["f16_gather_4x1"] = timeit(M, K, row, col, val, 32, "f16", 4, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
