"""ctypes bridge to the CPU oracle (oracle/liboracle_gs.so).

Test infrastructure: the oracle is only ever the checker."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle_gs.so")

OR_MAX_ARRAYS = 128
OR_NAME_LEN = 96


class OrArray(ctypes.Structure):
    _fields_ = [("key", ctypes.c_char * OR_NAME_LEN), ("len", ctypes.c_uint64),
                ("is_float", ctypes.c_int), ("u", ctypes.POINTER(ctypes.c_uint64)),
                ("f", ctypes.POINTER(ctypes.c_double))]


class OrSet(ctypes.Structure):
    _fields_ = [("a", OrArray * OR_MAX_ARRAYS), ("n", ctypes.c_int), ("err", ctypes.c_char * 256)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "gs_oracle.c")
        if (not os.path.exists(LIB)) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        _lib = ctypes.CDLL(LIB)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        f32p = ctypes.POINTER(ctypes.c_float)
        f64p = ctypes.POINTER(ctypes.c_double)
        _lib.or_init_set.argtypes = [ctypes.POINTER(OrSet), ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_uint64, u64p, u64p, f32p]
        _lib.or_pipeline.argtypes = [ctypes.POINTER(OrSet), ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        _lib.or_set_free.argtypes = [ctypes.POINTER(OrSet)]
        for name, vt in (("or_spmm_ref_f32", f32p), ("or_spmm_ref_f16", f32p)):
            fn = getattr(_lib, name)
            fn.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p, f32p, vt, vt]
        _lib.or_spmm_f64.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p,
                                     f32p, f64p, f64p]
        _lib.or_round_half.argtypes = [ctypes.c_float]
        _lib.or_round_half.restype = ctypes.c_float
        _lib.or_time_cpu_path.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p,
                                          f32p, ctypes.c_uint64, f64p, f64p]
        _lib.or_time_spmm_repeated.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p,
                                               f32p, ctypes.c_uint64, ctypes.c_double, f64p,
                                               ctypes.POINTER(ctypes.c_int)]
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def run_pipeline(M, K, row, col, val, pipeline, p0=0, p1=0):
    """Returns (dict key -> np.ndarray, error string or None)."""
    L = lib()
    row = np.ascontiguousarray(row, dtype=np.uint64)
    col = np.ascontiguousarray(col, dtype=np.uint64)
    val = np.ascontiguousarray(val, dtype=np.float32)
    s = OrSet()
    rc = L.or_init_set(ctypes.byref(s), M, K, len(row), _p(row, ctypes.c_uint64),
                       _p(col, ctypes.c_uint64), _p(val, ctypes.c_float))
    if rc == 0:
        rc = L.or_pipeline(ctypes.byref(s), pipeline.encode(), p0, p1)
    if rc != 0:
        err = s.err.decode()
        L.or_set_free(ctypes.byref(s))
        return None, err or "error"
    out = {}
    for i in range(s.n):
        a = s.a[i]
        n = a.len
        if a.is_float:
            out[a.key.decode()] = np.ctypeslib.as_array(a.f, shape=(n,)).copy() if n else np.zeros(0)
        else:
            out[a.key.decode()] = np.ctypeslib.as_array(a.u, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
    L.or_set_free(ctypes.byref(s))
    return out, None


def spmm_ref(M, N, row, col, val, B, mode="f32"):
    """CPU SpMM on the original COO.  mode: f32 | f16 (reference DType
    accumulation, kernel_lib.hpp:859-881) | f64."""
    L = lib()
    row = np.ascontiguousarray(row, dtype=np.uint64)
    col = np.ascontiguousarray(col, dtype=np.uint64)
    val = np.ascontiguousarray(val, dtype=np.float32)
    if mode == "f64":
        Bd = np.ascontiguousarray(B, dtype=np.float64)
        C = np.zeros((M, N), np.float64)
        L.or_spmm_f64(M, N, len(row), _p(row, ctypes.c_uint64), _p(col, ctypes.c_uint64),
                      _p(val, ctypes.c_float), _p(Bd, ctypes.c_double), _p(C, ctypes.c_double))
        return C
    Bf = np.ascontiguousarray(B, dtype=np.float32)
    C = np.zeros((M, N), np.float32)
    fn = L.or_spmm_ref_f32 if mode == "f32" else L.or_spmm_ref_f16
    fn(M, N, len(row), _p(row, ctypes.c_uint64), _p(col, ctypes.c_uint64),
       _p(val, ctypes.c_float), _p(Bf, ctypes.c_float), _p(C, ctypes.c_float))
    return C


def time_cpu_path(M, K, row, col, val, N):
    L = lib()
    row = np.ascontiguousarray(row, dtype=np.uint64)
    col = np.ascontiguousarray(col, dtype=np.uint64)
    val = np.ascontiguousarray(val, dtype=np.float32)
    t1 = ctypes.c_double()
    t2 = ctypes.c_double()
    rc = L.or_time_cpu_path(M, K, len(row), _p(row, ctypes.c_uint64), _p(col, ctypes.c_uint64),
                            _p(val, ctypes.c_float), N, ctypes.byref(t1), ctypes.byref(t2))
    if rc != 0:
        raise RuntimeError("oracle cpu path failed")
    return t1.value, t2.value


def time_spmm_repeated_mt(M, K, row, col, val, N, min_s, threads):
    """the build's all-cores host SpMM (OpenMP over rows) repeated for >= min_s seconds"""
    L = lib()
    L.or_time_spmm_repeated_mt.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_float), ctypes.c_uint64, ctypes.c_double,
                                           ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int)]
    row = np.ascontiguousarray(row, dtype=np.uint64)
    col = np.ascontiguousarray(col, dtype=np.uint64)
    val = np.ascontiguousarray(val, dtype=np.float32)
    t = ctypes.c_double()
    r = ctypes.c_int()
    rc = L.or_time_spmm_repeated_mt(M, K, len(row), _p(row, ctypes.c_uint64), _p(col, ctypes.c_uint64),
                                    _p(val, ctypes.c_float), N, min_s, int(threads), ctypes.byref(t), ctypes.byref(r))
    if rc != 0:
        raise RuntimeError("oracle cpu path failed")
    return t.value, r.value


def time_spmm_repeated(M, K, row, col, val, N, min_s):
    """host fp32 SpMM repeated for >= min_s seconds: (seconds, repetitions)"""
    L = lib()
    row = np.ascontiguousarray(row, dtype=np.uint64)
    col = np.ascontiguousarray(col, dtype=np.uint64)
    val = np.ascontiguousarray(val, dtype=np.float32)
    t = ctypes.c_double()
    r = ctypes.c_int()
    rc = L.or_time_spmm_repeated(M, K, len(row), _p(row, ctypes.c_uint64), _p(col, ctypes.c_uint64),
                                 _p(val, ctypes.c_float), N, min_s, ctypes.byref(t), ctypes.byref(r))
    if rc != 0:
        raise RuntimeError("oracle cpu path failed")
    return t.value, r.value


KINDS = {0: "none", 1: "linear", 2: "branch", 3: "cycle_linear", 4: "cycle_increase", 5: "residual"}


def index_compression(a, type_ori=16, branch_max=5):
    """oracle restatement of the reference's index-compression decision:
    (kind, {coef, intercept, cycle, aa, bb}, residual array or None)"""
    L = lib()
    a = np.ascontiguousarray(a, dtype=np.uint64)
    kind = ctypes.c_int(0)
    prm = np.zeros(5, np.uint64)
    res = np.zeros(max(1, len(a)), np.uint64)
    rc = L.or_index_compression(_p(a, ctypes.c_uint64), ctypes.c_uint64(len(a)), int(type_ori), int(branch_max),
                                ctypes.byref(kind), _p(prm, ctypes.c_uint64), _p(res, ctypes.c_uint64))
    assert rc == 0
    k = KINDS[kind.value]
    p = {"coef": int(prm[0]), "intercept": int(prm[1]), "cycle": int(prm[2]),
         "aa": int(prm[3].astype(np.int64)), "bb": int(prm[4].astype(np.int64))}
    return k, p, (res[:len(a)] if k == "residual" else None)
