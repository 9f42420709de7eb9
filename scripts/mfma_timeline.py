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
    plan.spmm(B, out=C) if "out" in plan.spmm.__code__.co_varnames else plan.spmm(B)
torch.cuda.synchronize()
L = _lib.load()
nb = int(M / 20)
st = (ctypes.c_uint64 * (nb * 64))()
_lib.check(L.gs_debug_mfma_timeline(plan._h, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), N,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), st, nb * 64))
a = np.frombuffer(st, dtype=np.uint64).reshape(nb, 64).astype(np.int64)
nc = info["lds_chunks"]
idx = [0, 1, 2, 3] + [4 + 5 * j + p for j in range(nc) for p in range(5)] + [63]
names = ["start", "loads0-2", "barrier0", "stage0"] + [f"c{j}.{p}" for j in range(nc)
                                                       for p in ("top", "ld+clr", "mfma", "mid", "stage")] + ["end"]
rel = a[:, idx] - a[:, [0]]
d = np.diff(rel, axis=1)
med = np.median(d, axis=0)
out = {"total_med": float(np.median(rel[:, -1])), "total_max": float(rel[:, -1].max()),
       "start_spread": float(a[:, 0].max() - a[:, 0].min()),
       "phases": {names[i + 1]: float(med[i]) for i in range(len(med))}}
print(json.dumps(out))
