"""generalsparse_amd -- MI355X-native SpMM (C = sparse_A x dense_B) behind
GeneralSparse's operator / plan surface.

Host-side mirror of the reference interface, over the C ABI of
libgeneralsparse.so (include/generalsparse.h):

    plan = Plan.from_mtx("m.mtx")                  # create_init_metadata_set_from_file
    plan.add_operator("sort_operator")              # operator_executer::add_and_run
    plan.add_operator("fixed_interval_row_direction_thread_blocking_operator",
                      1, 0, 0, 0, 0, 1, 4)
    plan.add_operator("thread_total_reduce_operator", 0, 4, 1)
    plan.compile()                                  # code_generator::compile
    plan.upload(dtype="f16")
    C = plan.spmm(B)                                # the generated kernel, on the GPU

or the canned token_test pipelines: plan.run_pipeline("warp_segment", N=32).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import GS_F16, GS_F32, GsError

__all__ = ["Plan", "Batch", "Rotation", "set_config", "GsError", "GS_F16", "GS_F32", "PIPELINES", "load_library"]

# token_test.cc pipelines (+ the two compositions this engine adds)
PIPELINES = ("thread_total", "warp_total", "block_total", "thread_bit_map", "warp_segment",
             "tblock_warp_total", "balanced_warp_total", "warp_bit_map", "tblock_bit_map", "col_direction_nm")


def load_library():
    return _lib.load()


def set_config(key, value):
    """set_config (config.cc:17-40); process-wide, in memory."""
    L = _lib.load()
    _lib.check(L.gs_set_config_int(key.encode(), int(value)))


def get_config(key):
    """the current value of an integer / bool config key"""
    L = _lib.load()
    v = ctypes.c_longlong()
    _lib.check(L.gs_get_config_int(key.encode(), ctypes.byref(v)))
    return v.value


def _dtype_code(dtype):
    if dtype in (GS_F16, "f16", "fp16", "half", np.float16):
        return GS_F16
    if dtype in (GS_F32, "f32", "fp32", "float", np.float32):
        return GS_F32
    try:
        import torch
        if dtype == torch.float16:
            return GS_F16
        if dtype == torch.float32:
            return GS_F32
    except ImportError:
        pass
    raise ValueError(f"unsupported dtype {dtype}")


def index_compression_of_array(a, type_ori=16, branch_max=5):
    """the reference's compression decision for a raw u64 array: (kind, {coef, intercept,
    cycle, aa, bb}, exact); type_ori = the gs data_type code of its storage (16 = u64)"""
    L = _lib.load()
    a = np.ascontiguousarray(a, dtype=np.uint64)
    kind = ctypes.create_string_buffer(32)
    prm = np.zeros(5, np.uint64)
    ex = ctypes.c_int(0)
    _lib.check(L.gs_index_compression_of_array(a.ctypes.data_as(_lib.u64p), len(a), int(type_ori), int(branch_max), kind, 32,
                                               prm.ctypes.data_as(_lib.u64p), ctypes.byref(ex)))
    p = {"coef": int(prm[0]), "intercept": int(prm[1]), "cycle": int(prm[2]),
         "aa": int(prm[3].astype(np.int64)), "bb": int(prm[4].astype(np.int64))}
    return kind.value.decode(), p, bool(ex.value)


def _refused(msg):
    """the error the library raises for a refused argument (GS_ERR code -1)"""
    e = GsError(f"generalsparse error -1: {msg}")
    e.code = -1
    return e


def _check_operands(info, B, C, N=None):
    """B (cols x N) and C (rows x N): contiguous GPU tensors of the plan's dtype on one device.
    The kernels read B and write every row of C at stride N, so a short or strided operand would
    be read or written out of bounds; raw pointers (ints) are the caller's responsibility."""
    import torch
    want = torch.float16 if info["dtype"] == GS_F16 else torch.float32
    if not (B.is_cuda and B.dim() == 2 and B.is_contiguous()):
        raise ValueError("B must be a contiguous 2-D GPU tensor")
    if B.shape[0] != info["cols"]:
        raise ValueError(f"B has {B.shape[0]} rows, A has {info['cols']} columns")
    if B.dtype != want:
        raise TypeError(f"B must be {want}")
    N = B.shape[1] if N is None else N
    if B.shape[1] != N:
        raise ValueError(f"B has {B.shape[1]} columns, expected {N}")
    if C is not None and not (C.is_cuda and C.device == B.device and C.is_contiguous() and C.dtype == want
                              and tuple(C.shape) == (info["rows"], N)):
        raise ValueError(f"C must be a contiguous {want} tensor of shape ({info['rows']}, {N}) on {B.device}")
    return want, N


class Batch:
    """a fixed list of SpMMs (plan, replica, B, C) run by gs_spmm_batch: consecutive K-split
    matrix-core entries of one instantiation are one grouped launch (k_mfma_ks_group).  The
    argument arrays are built once; run() enqueues the whole batch on a stream."""

    def __init__(self, entries, N):
        self._L = _lib.load()
        n = len(entries)
        self.plans = [e[0] for e in entries]  # keeps the plans alive
        for e in entries:
            if not isinstance(e[2], int):
                _check_operands(e[0].info(), e[2], None if isinstance(e[3], int) else e[3], int(N))
        self._p = (ctypes.c_void_p * n)(*[e[0]._h for e in entries])
        self._r = (ctypes.c_int * n)(*[int(e[1]) for e in entries])
        self._b = (ctypes.c_void_p * n)(*[e[2] if isinstance(e[2], int) else e[2].data_ptr() for e in entries])
        self._c = (ctypes.c_void_p * n)(*[e[3] if isinstance(e[3], int) else e[3].data_ptr() for e in entries])
        self.n, self.N = n, int(N)

    def run(self, stream=0):
        _lib.check(self._L.gs_spmm_batch(self._p, self._r, self._b, self._c, self.n, self.N, ctypes.c_void_p(stream)))

    def launches(self):
        """entries per launch, as run() enqueues them (gs_batch_launches): a grouped
        k_mfma_ks_group launch carries up to 32 entries"""
        cap = max(1, self.n)
        out = (ctypes.c_int * cap)()
        k = self._L.gs_batch_launches(self._p, self._r, self.n, self.N, out, cap)
        if k < 0:
            _lib.check(k)
        return [out[i] for i in range(min(k, cap))]


class Rotation:
    """`count` SpMMs of one plan from native code (gs_spmm_rotate), rotating its replicas and
    a fixed list of (B, C) pairs: launch i uses pair (first + i) % len(Bs).  The operands are
    checked and the pointer arrays built here, once, so run() adds only the native call."""

    def __init__(self, plan, Bs, Cs):
        n = len(Bs)
        if n == 0 or len(Cs) != n:
            raise ValueError("Bs and Cs must be non-empty lists of one length")
        info = plan.info()
        self.N = int(Bs[0].shape[1])
        for b, c in zip(Bs, Cs):
            _check_operands(info, b, c, self.N)
        self.plan, self.Bs, self.Cs, self.n = plan, Bs, Cs, n  # keeps plan and operands alive
        self._bp = (ctypes.c_void_p * n)(*[b.data_ptr() for b in Bs])
        self._cp = (ctypes.c_void_p * n)(*[c.data_ptr() for c in Cs])
        self._dev = Bs[0].device

    def run(self, count, first=0, stream=None):
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(self._dev).cuda_stream
        _lib.check(self.plan._L.gs_spmm_rotate(self.plan._h, int(count), int(first), self._bp, self._cp, self.n,
                                               self.N, ctypes.c_void_p(stream)))


class Plan:
    """A GeneralSparse plan: metadata set + operator history + code generator +
    device copies.  Wraps gs_plan_t."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        self._L = _lib.load()

    # ---------------------------------------------------------------- create
    @classmethod
    def from_mtx(cls, path, ones_values=True):
        """Reference reader semantics by default: every value := 1 (struct.cc:186-200)."""
        L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(L.gs_plan_create_from_mtx(str(path).encode(), int(bool(ones_values)), ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def load(cls, path):
        """a compiled plan from a binary plan file (plan_io.cc); upload() before spmm()"""
        L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(L.gs_plan_load(str(path).encode(), ctypes.byref(h)))
        return cls(h.value)

    def save(self, path):
        """writes the compiled plan (kernel selection + every plan array) to one binary file"""
        _lib.check(self._L.gs_plan_save(self._h, str(path).encode()))
        return self

    @classmethod
    def from_coo(cls, n_rows, n_cols, row, col, val=None):
        """Row-sorted COO; the dims grow to the largest index + 1 (the reference derives them
        from the entries, struct.cc:104-131).  row / col / val must hold the same number of
        entries and the indices must be non-negative integers."""
        L = _lib.load()
        row, col = np.asarray(row), np.asarray(col)
        for name, a in (("row", row), ("col", col)):
            if a.ndim != 1 or (a.size and not np.issubdtype(a.dtype, np.integer)):
                raise _refused(f"from_coo: {name} must be a 1-D integer array")
            if a.size and a.min() < 0:
                raise _refused(f"from_coo: negative {name} index")
        if len(col) != len(row) or (val is not None and len(val) != len(row)):
            raise _refused("from_coo: row, col and val lengths differ")
        row = np.ascontiguousarray(row, dtype=np.uint64)
        col = np.ascontiguousarray(col, dtype=np.uint64)
        vp = None
        if val is not None:
            val = np.ascontiguousarray(val, dtype=np.float32)
            vp = val.ctypes.data_as(_lib.f32p)
        h = ctypes.c_void_p()
        _lib.check(L.gs_plan_create_from_coo(int(n_rows), int(n_cols), len(row), row.ctypes.data_as(_lib.u64p),
                                             col.ctypes.data_as(_lib.u64p), vp, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def from_scipy(cls, A):
        A = A.tocsr()
        A.sort_indices()
        coo = A.tocoo()
        return cls.from_coo(A.shape[0], A.shape[1], coo.row, coo.col, coo.data)

    # ------------------------------------------------------------ operators
    def add_operator(self, name, *args, sub=0):
        """operator_executer::add_and_run of the named operator on sub-matrix `sub`
        (the reference's code_generator(meta, sub) target)"""
        arr = (ctypes.c_longlong * max(1, len(args)))(*[int(a) for a in args])
        _lib.check(self._L.gs_plan_add_operator_sub(self._h, int(sub), name.encode(), arr, len(args)))
        return self

    def run_pipeline(self, name, N, p0=0, p1=0, sub=0):
        _lib.check(self._L.gs_plan_run_pipeline_sub(self._h, int(sub), name.encode(), int(N), int(p0), int(p1)))
        return self

    def divide_rows(self, interval, sub=0):
        """fixed_interval_row_matrix_div_operator: one new sub-matrix per non-empty interval
        of `interval` rows; returns the live sub-matrix ids"""
        self.add_operator("fixed_interval_row_matrix_div_operator", int(interval), sub=sub)
        return self.sub_matrices()

    def sub_matrices(self):
        n = self._L.gs_plan_sub_matrices(self._h, None, 0)
        _lib.check(min(n, 0))
        ids = (ctypes.c_int * max(1, n))()
        _lib.check(min(self._L.gs_plan_sub_matrices(self._h, ids, n), 0))
        return list(ids[:n])

    def compile(self):
        _lib.check(self._L.gs_plan_compile(self._h))
        return self

    def generate_program(self, root, repeat=100):
        buf = ctypes.create_string_buffer(4096)
        _lib.check(self._L.gs_plan_generate_program(self._h, str(root).encode(), int(repeat), buf, 4096))
        return buf.value.decode()

    # --------------------------------------------------------------- device
    def upload(self, dtype="f16", device=0):
        self.dtype_code = _dtype_code(dtype)
        _lib.check(self._L.gs_plan_upload(self._h, self.dtype_code, int(device)))
        return self

    def add_replica(self):
        _lib.check(self._L.gs_plan_add_replica(self._h))

    def spmm(self, B, C=None, replica=0, stream=None):
        """C = A @ B on the GPU.  B: (K, N) torch tensor on the plan's device, in
        the plan's dtype.  Enqueued on torch's current stream."""
        import torch
        info = self.info()
        want, N = _check_operands(info, B, C)
        if C is None:
            C = torch.empty((info["rows"], N), dtype=want, device=B.device)
        s = stream if stream is not None else torch.cuda.current_stream(B.device).cuda_stream
        _lib.check(self._L.gs_spmm_replica(self._h, int(replica), ctypes.c_void_p(B.data_ptr()),
                                           ctypes.c_void_p(C.data_ptr()), int(N), ctypes.c_void_p(s)))
        return C

    def rotation(self, Bs, Cs):
        """the (B, C) pairs of spmm_rotate, checked and packed once; .run(count, first) enqueues"""
        return Rotation(self, Bs, Cs)

    def spmm_rotate(self, count, first, Bs, Cs, stream=None):
        """`count` SpMMs from native code, rotating replicas and the (B, C) pairs."""
        self.rotation(Bs, Cs).run(count, first, stream)

    def spmm_raw(self, B_ptr, C_ptr, N, replica=0, stream=0):
        _lib.check(self._L.gs_spmm_replica(self._h, int(replica), ctypes.c_void_p(B_ptr), ctypes.c_void_p(C_ptr),
                                           int(N), ctypes.c_void_p(stream)))

    # ------------------------------------------------------------ inspection
    def info(self):
        i = _lib.GsPlanInfo()
        _lib.check(self._L.gs_plan_info_get(self._h, ctypes.byref(i)))
        return {k: (getattr(i, k).decode() if k in ("kernel_name", "device_kernel") else getattr(i, k))
                for k, _ in i._fields_}

    def keys(self):
        n = self._L.gs_plan_array_count(self._h)
        out = []
        buf = ctypes.create_string_buffer(256)
        for i in range(n):
            _lib.check(self._L.gs_plan_array_key(self._h, i, buf, 256))
            out.append(buf.value.decode())
        return out

    def array(self, key):
        k = key.encode()
        n = self._L.gs_plan_array_len(self._h, k)
        if n < 0:
            raise KeyError(key)
        if self._L.gs_plan_array_is_float(self._h, k) == 1:
            a = np.zeros(n, np.float64)
            _lib.check(self._L.gs_plan_array_read_f64(self._h, k, a.ctypes.data_as(_lib.f64p), n))
        else:
            a = np.zeros(n, np.uint64)
            _lib.check(self._L.gs_plan_array_read_u64(self._h, k, a.ctypes.data_as(_lib.u64p), n))
        return a

    def arrays(self):
        return {k: self.array(k) for k in self.keys()}

    def index_compression(self, key):
        """(kind, expression of i, exact) for one integer plan array (code_generator.cc:2618-3063;
        "none" unless MODEL_DRIVEN_COMPRESS is set)"""
        kind = ctypes.create_string_buffer(32)
        expr = ctypes.create_string_buffer(1 << 14)
        ex = ctypes.c_int(0)
        _lib.check(self._L.gs_plan_index_compression(self._h, key.encode(), kind, 32, expr, 1 << 14, ctypes.byref(ex)))
        return kind.value.decode(), expr.value.decode(), bool(ex.value)

    def logical_check(self):
        """"" when the metadata set is consistent, else the first violation
        (logical_check, metadata_set.cc:806-1890)"""
        buf = ctypes.create_string_buffer(1024)
        rc = self._L.gs_plan_logical_check(self._h, buf, 1024)
        _lib.check(min(rc, 0))
        return buf.value.decode()

    def set_array_entry(self, key, i, value):
        """metadata editing (tools / tests): entry i of an integer plan array"""
        _lib.check(self._L.gs_plan_array_set_u64(self._h, key.encode(), int(i), int(value)))
        return self

    def device_status(self, stream=0):
        """synchronises `stream` and raises GsError (code GS_ERR_DEVICE) if a launch of this
        plan reported a device fault since the last call (gs_plan_device_status: a K-split
        combine that gave up waiting for a partial slab)"""
        _lib.check(self._L.gs_plan_device_status(self._h, ctypes.c_void_p(stream)))
        return self

    def log(self):
        buf = ctypes.create_string_buffer(1 << 16)
        _lib.check(self._L.gs_plan_log(self._h, buf, 1 << 16))
        return buf.value.decode()

    def free(self):
        if self._h is not None and self._h.value:
            self._L.gs_plan_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
