"""Phase timeline of k_mfma_ks on C2 (diagnostic: gs_debug_mfma_timeline on a k_mfma_ks plan).
Per slot: median / p90 over waves of s_memtime - the workgroup's first stamp (shader clocks).
Slots: 0 start, 1 loads issued, 2 after B barrier, 3+i after step i, 20 loop done, 21 reduced, 22 end."""
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

M = int(os.environ.get("TL_M", "5120"))  # TL_M / TL_K: another shape (attn: 7168)
K = int(os.environ.get("TL_K", str(M)))
N = 32
P0 = int(sys.argv[1]) if len(sys.argv) > 1 else 80
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
gsa.set_config("KS_PRIO", int(os.environ.get("KS_PRIO", "1")))
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, P0, 1).compile().upload("f16", 0)
info = plan.info()
B = torch.randn((K, N), device="cuda", dtype=torch.float16)
C = torch.empty((M, N), device="cuda", dtype=torch.float16)
for _ in range(50):
    plan.spmm(B)
torch.cuda.synchronize()
L = _lib.load()
nwg = (M + P0 - 1) // P0 * info["ksplit"]
n = nwg * 8 * 32
st = (ctypes.c_uint64 * n)()
_lib.check(L.gs_debug_mfma_timeline(plan._h, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), N,
                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), st, n))
a = np.frombuffer(st, dtype=np.uint64).reshape(nwg, 8, 32).astype(np.int64)
t0 = a[:, :, 0].min(axis=1)[:, None]
glob0 = a[:, :, 0].min()
# s_memtime is per XCD (clocks of different XCDs are not aligned): every delta is taken
# inside one workgroup (from its first stamp)
out = {"M": M, "K": K, "ksplit": info["ksplit"], "rows": P0}
for slot in [1, 2] + list(range(3, 16)) + [20, 21, 22]:
    v = a[:, :, slot]
    ok = v > 0
    if not ok.any():
        continue
    d = (v - t0)[ok]
    out[str(slot)] = [float(np.median(d)), float(np.percentile(d, 90)), int(ok.sum())]
# per wave index: loop done (slot 20) relative to the workgroup's first stamp
out["loop_done_by_wave"] = [float(np.median(a[:, w, 20] - t0[:, 0])) for w in range(a.shape[1])]
out["step0_by_wave"] = [float(np.median(a[:, w, 3] - t0[:, 0])) for w in range(a.shape[1])]
# spread of loop-done inside a workgroup (max - min over its waves)
ld = a[:, :, 20] - t0
out["loop_done_spread_in_wg"] = [float(np.median(ld.max(axis=1) - ld.min(axis=1))), float(np.percentile(ld.max(axis=1) - ld.min(axis=1), 90))]
span = a[:, :, 22].max(axis=1) - t0[:, 0]
out["wg_span_clk"] = [float(np.median(span)), float(np.percentile(span, 90)), float(span.max())]
print(json.dumps(out))
