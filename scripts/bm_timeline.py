"""Phase timeline of k_mfma_bm on C2 (diagnostic: gs_debug_mfma_timeline on a k_mfma_bm plan,
80-row blocks, 8 waves).  Per slot: median / p90 over waves of s_memtime - the launch's first
stamp (shader clocks, 100 MHz on gfx950's s_memtime?  printed raw), plus the spread of
workgroup starts.  Slots: 0 start, 1 B + records issued, 2 values issued, 3 B stored,
4 first batch's MFMAs done, 5 loop done, 6 reduced, 7 slab published, 8 end."""
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
P0 = int(sys.argv[1]) if len(sys.argv) > 1 else 80
gsa.set_config("MFMA_BM", 1)
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, P0, 1).compile().upload("f16", 0)
info = plan.info()
B = torch.randn((K, N), device="cuda", dtype=torch.float16)
C = torch.empty((M, N), device="cuda", dtype=torch.float16)
for _ in range(200):
    plan.spmm(B)
torch.cuda.synchronize()
L = _lib.load()
nwg = (M + P0 - 1) // P0 * info["ksplit"]
n = nwg * 8 * 16
st = (ctypes.c_uint64 * n)()
_lib.check(L.gs_debug_mfma_timeline(plan._h, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), N,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), st, n))
a = np.frombuffer(st, dtype=np.uint64).reshape(nwg, 8, 16).astype(np.int64)
glob0 = a[:, :, 0].min()
out = {"ksplit": info["ksplit"], "kernel": info["device_kernel"],
       "wg_start_spread": [float(np.percentile(a[:, :, 0].min(axis=1) - glob0, p)) for p in (0, 50, 90, 100)]}
for slot in range(1, 9):
    v = a[:, :, slot]
    ok = v > 0
    if not ok.any():
        continue
    d = (v - glob0)[ok]
    out[str(slot)] = [float(np.median(d)), float(np.percentile(d, 90)), float(d.max()), int(ok.sum())]
print(json.dumps(out))
