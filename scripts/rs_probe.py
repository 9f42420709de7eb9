import ctypes, os, sys, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
from generalsparse_amd import datasets as ds
lib = ctypes.CDLL(os.path.join("generalsparse_amd", "librocsparse_cmp.so"))
lib.rs_last_error.restype = ctypes.c_char_p
M = K = 5120; N = 32
row, col, val = ds.pruned_weight(M, K, 0.7, 13)
rp = np.zeros(M + 1, np.int64); np.add.at(rp, row.astype(np.int64) + 1, 1); rp = np.cumsum(rp).astype(np.int32)
c32 = col.astype(np.int32); v = val.astype(np.float32)
out = {}
for dtype in (1, 0):
    for alg in (0, 1, 4, 5, 9):
        ms = ctypes.c_double()
        rc = lib.rs_spmm_bench(M, K, len(v), rp.ctypes.data_as(ctypes.c_void_p), c32.ctypes.data_as(ctypes.c_void_p),
                               v.ctypes.data_as(ctypes.c_void_p), N, dtype, alg, 5, 50, 16, ctypes.byref(ms), None)
        out[f"dt{dtype}_alg{alg}"] = (rc, ms.value, lib.rs_last_error().decode() if rc else "",
                                      2.0 * len(v) * N / (ms.value * 1e-3) / 1e9 if rc == 0 else None)
print(json.dumps(out, indent=0))
