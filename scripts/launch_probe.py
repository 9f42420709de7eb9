"""Where the C2 step time goes between launches (diagnostic): host enqueue cost of
spmm_rotate, HIP-event time on one stream, the same launches captured in a HIP graph, and
launches alternating over two streams (independent SpMMs).  usage: launch_probe.py [p0] [steps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

P0 = int(sys.argv[1]) if len(sys.argv) > 1 else 40
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
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


def ev(fn, stream=None):
    s = stream or torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    t0 = time.perf_counter()
    fn()
    t_host = time.perf_counter() - t0
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / STEPS, t_host * 1e6 / STEPS


plan.spmm_rotate(500, 0, Bs, Cs)
res = []
for _ in range(3):
    res.append(ev(lambda: plan.spmm_rotate(STEPS, 0, Bs, Cs)))
out["one_stream_us"] = [round(r[0], 3) for r in res]
out["host_enqueue_us_per_launch"] = [round(r[1], 3) for r in res]
# launches one at a time from Python (the per-call ctypes path)
res = []
for _ in range(2):
    bp = [b.data_ptr() for b in Bs]
    cp = [c.data_ptr() for c in Cs]
    cs = torch.cuda.current_stream().cuda_stream
    res.append(ev(lambda: [plan.spmm_raw(bp[i % R], cp[i % R], N, i % R, cs) for i in range(STEPS)]))
out["one_stream_python_loop_us"] = [round(r[0], 3) for r in res]
out["python_loop_host_us_per_launch"] = [round(r[1], 3) for r in res]
# HIP graph of the same launches
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    plan.spmm_rotate(2, 0, Bs, Cs)
torch.cuda.synchronize()
with torch.cuda.graph(g, stream=s):
    plan.spmm_rotate(STEPS, 0, Bs, Cs)
g.replay()
torch.cuda.synchronize()
res = [ev(lambda: g.replay(), stream=s) for _ in range(3)]
out["graph_us"] = [round(r[0], 3) for r in res]
# two streams alternating (independent SpMMs: replica i, B/C i)
s2 = [torch.cuda.current_stream(), torch.cuda.Stream()]


def two():
    e = torch.cuda.Event()
    e.record(s2[0])
    s2[1].wait_event(e)
    for i in range(STEPS):
        plan.spmm_raw(Bs[i % R].data_ptr(), Cs[i % R].data_ptr(), N, i % R, s2[i % 2].cuda_stream)
    e2 = torch.cuda.Event()
    e2.record(s2[1])
    s2[0].wait_event(e2)


res = [ev(two) for _ in range(3)]
out["two_streams_us"] = [round(r[0], 3) for r in res]
print(json.dumps(out))
