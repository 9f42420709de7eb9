"""C2 plan sweep (diagnostic): rows per BMTB x K-split for the matrix-core kernel,
kernel time by HIP events over rotated replicas.  usage: c2_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

M = K = 5120
N = 32
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
for pipe, rb, wb in [("tblock_warp_total", 20, 2), ("block_total", 20, 1), ("block_total", 32, 1),
                     ("block_total", 40, 1), ("block_total", 64, 1), ("block_total", 80, 1)]:
    for ks in (1, 2, 4):
        gsa.set_config("MFMA_KSPLIT", ks)
        try:
            plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, rb, wb).compile().upload("f16", 0)
        except Exception as ex:
            print(pipe, rb, ks, "error", ex)
            continue
        info = plan.info()
        reps = 12
        for _ in range(reps - 1):
            plan.add_replica()
        Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
        Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
        plan.spmm_rotate(20, 0, Bs, Cs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.spmm_rotate(200, 0, Bs, Cs)
        e1.record()
        torch.cuda.synchronize()
        print(f"{pipe}({rb},{wb}) ks={ks} lds_stage={info['lds_stage']} ksplit={info.get('ksplit')} "
              f"kernel_us={e0.elapsed_time(e1) / 200 * 1e3:.2f}", flush=True)
        plan.free()
gsa.set_config("MFMA_KSPLIT", 0)
