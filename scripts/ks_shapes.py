"""k_mfma_ks vs k_mfma_rows on the C5 shapes (diagnostic): event time per launch with rotated replicas.
usage: ks_shapes.py [sparsity]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402
from ks_check import timeit  # noqa: E402

sp = float(sys.argv[1]) if len(sys.argv) > 1 else 0.8
shapes = {"attn": (7168, 7168), "fc1": (28672, 7168), "fc2": (7168, 28672)}
for name, (M, K) in shapes.items():
    row, col, val = ds.pruned_weight(M, K, sp, 7)
    cands = {"attn": [("tblock_warp_total", 28, 2, ()), ("block_total", 80, 1, ()), ("block_total", 56, 1, ()),
                      ("block_total", 64, 1, ())],
             "fc1": [("tblock_warp_total", 56, 2, ()), ("block_total", 80, 1, ()), ("block_total", 64, 1, ())],
             "fc2": [("tblock_warp_total", 28, 2, ()), ("block_total", 80, 1, ()), ("block_total", 56, 1, ()),
                     ("block_total", 80, 1, (("KS_SPLIT", 8),))]}[name]
    for (pipe, p0, p1, cfg) in cands:
        print(name, end=" ")
        timeit(M, K, 32, row, col, val, pipe, p0, p1, cfg)
