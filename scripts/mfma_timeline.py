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
P0 = int(sys.argv[1]) if len(sys.argv) > 1 else 20  # rows per BMTB
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, P0, 1).compile().upload("f16", 0)
info = plan.info()
B = torch.randn((K, N), device="cuda", dtype=torch.float16)
C = torch.empty((M, N), device="cuda", dtype=torch.float16)
for _ in range(20):
    plan.spmm(B)
torch.cuda.synchronize()
L = _lib.load()
nb = (M + P0 - 1) // P0 * info["ksplit"]
st = (ctypes.c_uint64 * (nb * 64))()
_lib.check(L.gs_debug_mfma_timeline(plan._h, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), N,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), st, nb * 64))
a = np.frombuffer(st, dtype=np.uint64).reshape(nb, 64).astype(np.int64)
nc = (info["lds_chunks"] + info["ksplit"] - 1) // info["ksplit"]
t0 = a[:, [0]]
out = {"total_med": float(np.median(a[:, 63] - a[:, 0])), "total_max": float((a[:, 63] - a[:, 0]).max())}
# slot layout (kernel_lib.hpp k_mfma_rows STAMPS): role r (0 compute, 1 B rows, 2 entries) in
# slots 21r..21r+20: 0 start, 1 chunk 0 staged, 2+2j chunk j's work done, 3+2j after its barrier
for name, r in (("compute", 0), ("bload", 1), ("aload", 2)):
    base = 21 * r
    rows = {"staged0": float(np.median(a[:, base + 1] - t0[:, 0]))}
    for j in range(min(nc, 9)):
        rows[f"c{j}"] = [float(np.median(a[:, base + 2 + 2 * j] - t0[:, 0])),
                         float(np.median(a[:, base + 3 + 2 * j] - t0[:, 0]))]
    out[name] = rows
print(json.dumps(out))
