"""Device index compression, measured: one gather-family plan with
MODEL_DRIVEN_COMPRESS off (argv[1] = 0) or on (1), launched `steps` times over rotated
replicas (A of all replicas > the 256 MB Infinity Cache), prints one JSON line with the
plan's device bytes, the formulas used and the average kernel time (HIP events on the
launch stream).  Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE for the HBM bytes
(scripts/gpu_compress.sh -> profiles/traffic_compression.json).

Workload: 4,000,000 rows x 60,000 columns, 4 nnz per row (seeded uniform rows), fp16,
N = 8, tblock_warp_total(4, 1) on the gather kernel (k_warp_rows with BMTB grouping):
per row the kernel reads a CSR row pointer, a BMW row start and a quarter of a BMTB ->
BMW entry besides its 4 (u16 column, fp16 value) pairs -- the two plan arrays are
linear and become formulas."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402

compress = int(sys.argv[1]) if len(sys.argv) > 1 else 1
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
M, K, NPR, N = 4_000_000, 60_000, 4, 8
rng = np.random.default_rng(5)
row = np.repeat(np.arange(M, dtype=np.uint64), NPR)
col = np.sort(rng.integers(0, K, (M, NPR)), axis=1).astype(np.uint64).ravel()
val = rng.uniform(-1, 1, M * NPR).astype(np.float32)
gsa.set_config("MFMA_TILES", 0)
gsa.set_config("LDS_STAGE_B", 0)
gsa.set_config("MODEL_DRIVEN_COMPRESS", compress)
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("tblock_warp_total", N, 4, 1).compile().upload("f16", 0)
gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)
info = plan.info()
reps = 4
for _ in range(reps - 1):
    plan.add_replica()
Bs = [torch.empty((K, N), device="cuda", dtype=torch.float16).uniform_(-1, 1) for _ in range(reps)]
Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(reps)]
plan.spmm_rotate(20, 0, Bs, Cs)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
plan.spmm_rotate(steps, 0, Bs, Cs, stream=s.cuda_stream)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / steps
# algorithmic bytes: A as the uncompressed plan stores it, B rows gathered once, C written once
alg_A_uncompressed = info["device_bytes_A"] + info["index_bytes_saved"]
print(json.dumps({"compress": compress, "device_kernel": info["device_kernel"], "device_bytes_A": info["device_bytes_A"],
                  "index_formulas": info["index_formulas"], "index_bytes_saved": info["index_bytes_saved"],
                  "kernel_ms": round(ms, 5), "steps": steps, "replicas": reps,
                  "A_bytes_uncompressed": alg_A_uncompressed, "C_bytes": M * N * 2, "B_bytes": K * N * 2}))
