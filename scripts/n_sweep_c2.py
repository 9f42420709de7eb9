"""C2 at several dense widths (diagnostic): every candidate plan, its kernel and event time
with rotated replicas; parity of the matrix-core kernels vs a torch fp32 product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ks_check import check, timeit  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

row, col, val = ds.pruned_weight(5120, 5120, 0.7, 13)
Ns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,16,32,64,128").split(",")]
for N in Ns:
    for (pipe, p0, p1) in [("tblock_warp_total", 20, 2), ("block_total", 40, 1), ("block_total", 64, 1),
                           ("block_total", 80, 1)]:
        if N in (8, 128):
            check(5120, 5120, N, row, col, val, pipe, p0, p1)
        print(f"N={N}", end=" ")
        timeit(5120, 5120, N, row, col, val, pipe, p0, p1)
