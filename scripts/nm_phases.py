"""C3 k_nm_mfma phase attribution (diagnostic; experiments build, GS_LIBRARY=...exp.so).
GS_NM_DEBUG=4: s_memtime stamps per half iteration (B staged to LDS / B loads issued / compute /
A loads issued / barrier passed) of waves 0 and 4 of workgroups 0 and 100, printed by the kernel;
GS_NM_DEBUG=1 / 2: the loop without B / A loads, 8: without the odd n-tiles' B fragment reads
(wrong results, timing only).
usage: GS_NM_DEBUG=<0|1|2|4|8> nm_phases.py [N] [launches]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
L = int(sys.argv[2]) if len(sys.argv) > 2 else 50
M, K = 28672, 7168
r, c, v = ds.two_four(M, K, 30)
gsa.set_config("NM_NT", 0)  # the stamp build runs the default-policy kernel
plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("col_direction_nm", N, 32, 1).compile().upload("f16", 0)
R = 8
for _ in range(R - 1):
    plan.add_replica()
Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(R)]
Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(R)]
dbg = os.environ.get("GS_NM_DEBUG", "0")
if dbg == "4":
    plan.spmm(Bs[0], C=Cs[0])
    torch.cuda.synchronize()
else:
    plan.spmm_rotate(10, 0, Bs, Cs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.spmm_rotate(L, 0, Bs, Cs)
    e1.record()
    torch.cuda.synchronize()
    print(f"GS_NM_DEBUG={dbg} N={N}: {e0.elapsed_time(e1) / L * 1e3:.2f} us per launch")
