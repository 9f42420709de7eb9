"""Phase timeline of k_mfma_rows on C2 (diagnostic: gs_debug_mfma_timeline).
Prints, per phase, the median over workgroups of the s_memtime delta from the
previous stamp (shader clocks), and the per-chunk totals."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import _lib  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

M = K = 5120
N = 32
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, 20, 1).compile().upload("f16", 0)
info = plan.info()
B = torch.randn((K, N), device="cuda", dtype=torch.float16)
C = torch.empty((M, N), device="cuda", dtype=torch.float16)
for _ in range(20):
    plan.spmm(B)
torch.cuda.synchronize()
L = _lib.load()
nb = int(M / 20)
st = (ctypes.c_uint64 * (nb * 64))()
_lib.check(L.gs_debug_mfma_timeline(plan._h, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), N,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), st, nb * 64))
a = np.frombuffer(st, dtype=np.uint64).reshape(nb, 64).astype(np.int64)
nc = info["lds_chunks"]
t0 = a[:, [0]]
out = {"total_med": float(np.median(a[:, 31] - a[:, 0])), "total_max": float((a[:, 31] - a[:, 0]).max())}
# slot layout (kernel_lib.hpp k_mfma_rows STAMPS): compute lane 0 in 0..30, loader lane 0 in 32..62;
# 0 start, 1 chunk 0 staged; per chunk j: 2+3j work done (loader: loads issued), 3+3j (loader: staged),
# 4+3j after the chunk's barrier; 31 end
for name, base in (("compute", 0), ("loader", 32)):
    rows = {"staged0": float(np.median(a[:, base + 1] - t0[:, 0]))}
    for j in range(min(nc, 9)):
        ph = [float(np.median(a[:, base + k + 3 * j] - t0[:, 0])) for k in (2, 3, 4)]
        rows[f"c{j}"] = ph
    out[name] = rows
print(json.dumps(out, indent=0))
