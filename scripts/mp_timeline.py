"""Phase timeline of k_merge_path on the C4 webbase-1M stand-in (diagnostic: the experiments
build, GS_LIBRARY=.../libgeneralsparse_exp.so, gs_debug_mfma_timeline on a merge-path plan).
Per slot: median / p90 over path waves of s_memtime - the wave's first stamp (shader clocks).
Slots: 1 first loads issued; per round r < 4: 2+3r gathers issued, 3+3r rows staged, 4+3r walked
and scanned; 14 loop done; 15 end.  usage: mp_timeline.py [work_size]"""
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

M, N = 1000005, 8
ws = int(sys.argv[1]) if len(sys.argv) > 1 else 512
row, col, val = ds.rmat(M, 3105536, 1)
plan = gsa.Plan.from_coo(M, M, row, col, val).run_pipeline("merge_path", N, ws, 1).compile().upload("f32", 0)
info = plan.info()
B = torch.randn((M, N), device="cuda", dtype=torch.float32)
C = torch.empty((M, N), device="cuda", dtype=torch.float32)
for _ in range(20):
    plan.spmm(B, C=C)
torch.cuda.synchronize()
L = _lib.load()
nw = info["n_units"]
n = nw * 16
st = (ctypes.c_uint64 * n)()
_lib.check(L.gs_debug_mfma_timeline(plan._h, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), N,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), st, n))
a = np.frombuffer(st, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
t0 = a[:, 0:1]
out = {"work_size": ws, "n_waves": int(nw)}
for slot in range(1, 16):
    v = a[:, slot]
    ok = v > 0
    if not ok.any():
        continue
    d = (v - t0[:, 0])[ok]
    out[str(slot)] = [float(np.median(d)), float(np.percentile(d, 90)), int(ok.sum())]
print(json.dumps(out))
