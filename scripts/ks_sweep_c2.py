"""C2 k_mfma_ks sweep (diagnostic): rows per BMTB x K ranges x waves, kernel time by HIP
events over rotated replicas (> 256 MB of A, past the Infinity Cache).
usage: ks_sweep_c2.py [rows,...] [splits,...] [waves,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

M = K = 5120
N = int(os.environ.get("SWEEP_N", "32"))
rows_l = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "40,64,80").split(",")]
spl_l = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,4,8").split(",")]
wav_l = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "8").split(",")]
prio_l = [int(x) for x in os.environ.get("SWEEP_PRIO", "1").split(",")]
KB = int(os.environ.get("SWEEP_KB", "0"))  # k_mfma_kb (bitmap layout; experiments build)
if KB:
    gsa.set_config("MFMA_BM", 1)
    gsa.set_config("BM_KB", 1)
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
for rb in rows_l:
    for ks in spl_l:
        for w, pr in [(w, pr) for w in wav_l for pr in prio_l]:
            gsa.set_config("KS_SPLIT", ks)
            gsa.set_config("BM_SPLIT", ks)
            gsa.set_config("KS_WAVES", w)
            gsa.set_config("KS_PRIO", pr)
            try:
                plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, rb, 1).compile().upload("f16", 0)
            except Exception as ex:
                print(json.dumps({"rows": rb, "split": ks, "waves": w, "prio": pr, "error": str(ex)}), flush=True)
                continue
            info = plan.info()
            reps = 12
            for _ in range(reps - 1):
                plan.add_replica()
            Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
            Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
            plan.spmm_rotate(40, 0, Bs, Cs)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                plan.spmm_rotate(200, 0, Bs, Cs)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 200 * 1e3)
            print(json.dumps({"rows": rb, "split": ks, "waves": w, "prio": pr, "kernel": info["device_kernel"],
                              "ksplit": info.get("ksplit"), "bytes_A": info.get("bytes_A"), "us": round(best, 2)}), flush=True)
            plan.free()
gsa.set_config("KS_SPLIT", 0)
gsa.set_config("KS_WAVES", 8)
gsa.set_config("KS_PRIO", 1)
