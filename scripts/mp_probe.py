"""C4 merge-path walk timing (diagnostic): event time of merge_path(ws, 1) on the webbase
stand-in with rotated replicas, under engine switches given as KEY=INT arguments.
usage: mp_probe.py [ws] [KEY=INT ...]   (GS_MP_DEBUG=4 in the environment: no in-launch combine)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402


def main():
    args = sys.argv[1:]
    ws = int(args[0]) if args and "=" not in args[0] else 512
    for kv in [a for a in args if "=" in a]:
        k, v = kv.split("=")
        gsa.set_config(k, int(v))
    M = 1000005
    row, col, val = ds.rmat(M, 3105536, 1, symmetric=False)  # bench.py c4 seed
    N = 8
    plan = gsa.Plan.from_coo(M, M, row, col, val).run_pipeline("merge_path", N, ws, 1).compile().upload("f32", 0)
    info = plan.info()
    nrep = 11
    for _ in range(nrep - 1):
        plan.add_replica()
    Bs = [torch.randn((M, N), device="cuda") for _ in range(nrep)]
    Cs = [torch.empty((M, N), device="cuda") for _ in range(nrep)]
    plan.spmm_rotate(200, 0, Bs, Cs)
    torch.cuda.synchronize()
    for rotate in (True, False):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if rotate:
            plan.spmm_rotate(300, 0, Bs, Cs)
        else:
            for _ in range(300):
                plan.spmm(Bs[0], C=Cs[0])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 300 * 1e3
        print(f"ws={ws} {' '.join(args)} GS_MP_DEBUG={os.environ.get('GS_MP_DEBUG', '0')} {info['device_kernel']} "
              f"units={info['n_units']} {'cold' if rotate else 'hot'} {us:.2f} us", flush=True)


if __name__ == "__main__":
    main()
