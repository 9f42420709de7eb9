"""C2 launches captured in a HIP graph (torch.cuda.CUDAGraph on a side stream) against the
same launches enqueued one by one (diagnostic): per-SpMM time by HIP events, and a check that
the replay wrote every C (each C NaN-filled before the replay, compared with the eager result).
usage: graph_probe.py [p0] [steps] [KEY=VALUE ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

for kv in [x for x in sys.argv[1:] if "=" in x]:
    k, v = kv.split("=", 1)
    gsa.set_config(k, int(v))
a = [x for x in sys.argv[1:] if "=" not in x]
P0 = int(a[0]) if len(a) > 0 else 40
STEPS = int(a[1]) if len(a) > 1 else 200
M = K = 5120
N = 32
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, P0, 1).compile().upload("f16", 0)
R = 20
for _ in range(R - 1):
    plan.add_replica()
Bs = [torch.randn((K, N), device="cuda", dtype=torch.float16) for _ in range(R)]
Cs = [torch.empty((M, N), device="cuda", dtype=torch.float16) for _ in range(R)]
out = {"plan": f"block_total({P0},1)", "kernel": plan.info()["device_kernel"], "steps": STEPS}


def ev(fn, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / STEPS, 3)


cur = torch.cuda.current_stream()
plan.spmm_rotate(100, 0, Bs, Cs)
out["eager_us"] = [ev(lambda: plan.spmm_rotate(STEPS, 0, Bs, Cs), cur) for _ in range(3)]
ref = [c.clone() for c in Cs]  # the last STEPS launches' outputs (every C written: STEPS >= R)
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
s.wait_stream(cur)
with torch.cuda.stream(s):
    plan.spmm_rotate(2, 0, Bs, Cs)
torch.cuda.synchronize()
with torch.cuda.graph(g, stream=s):
    for i in range(STEPS):
        plan.spmm_raw(Bs[i % R].data_ptr(), Cs[i % R].data_ptr(), N, i % R, s.cuda_stream)
for c in Cs:
    c.fill_(float("nan"))
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
out["graph_writes_every_C"] = all(bool(torch.equal(c, r)) for c, r in zip(Cs, ref))
out["graph_us"] = [ev(lambda: g.replay(), torch.cuda.current_stream()) for _ in range(3)]  # replay runs on the current stream
plan.device_status()
print(json.dumps(out))
