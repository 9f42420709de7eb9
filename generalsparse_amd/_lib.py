"""ctypes binding of include/generalsparse.h (libgeneralsparse.so, built in-tree).

The HIP extension is the product: if the library is missing this module raises
instead of falling back to any CPU path."""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# GS_LIBRARY: another build of the same library (e.g. the ASan/UBSan host build, make -C csrc san)
LIB_PATH = os.environ.get("GS_LIBRARY") or os.path.join(PKG_DIR, "libgeneralsparse.so")

GS_F32 = 0
GS_F16 = 1

u64p = ctypes.POINTER(ctypes.c_uint64)
f32p = ctypes.POINTER(ctypes.c_float)
f64p = ctypes.POINTER(ctypes.c_double)


class GsOpts(ctypes.Structure):
    _fields_ = [("pipeline", ctypes.c_char_p), ("dtype", ctypes.c_int), ("dense_n", ctypes.c_int),
                ("p0", ctypes.c_int), ("p1", ctypes.c_int), ("ones_values", ctypes.c_int),
                ("device", ctypes.c_int)]


class GsPlanInfo(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_uint64), ("cols", ctypes.c_uint64), ("nnz", ctypes.c_uint64),
                ("nnz_stored", ctypes.c_uint64), ("n_units", ctypes.c_uint64),
                ("device_bytes_A", ctypes.c_uint64), ("family", ctypes.c_int), ("col_bytes", ctypes.c_int),
                ("dtype", ctypes.c_int), ("replicas", ctypes.c_int), ("needs_memset", ctypes.c_int),
                ("kernel_name", ctypes.c_char * 64), ("lds_stage", ctypes.c_int), ("lds_n", ctypes.c_uint32),
                ("lds_kc", ctypes.c_uint32), ("lds_chunks", ctypes.c_uint32), ("lds_waves", ctypes.c_uint32),
                ("lds_bytes", ctypes.c_uint64), ("tile_bytes", ctypes.c_uint64), ("ksplit", ctypes.c_uint32),
                ("n_kernels", ctypes.c_int), ("device_kernel", ctypes.c_char * 32),
                ("index_formulas", ctypes.c_int), ("index_bytes_saved", ctypes.c_uint64),
                ("ks_nt", ctypes.c_uint32), ("ks_head_groups", ctypes.c_uint32),
                ("nm_tiles", ctypes.c_uint32)]


# every symbol include/generalsparse.h declares, with its ctypes signature
SIGNATURES = {
    "gs_plan_logical_check": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "gs_plan_array_set_u64": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64], ctypes.c_int),
    "gs_last_error": ([], ctypes.c_char_p),
    "gs_version": ([], ctypes.c_char_p),
    "gs_opts_default": ([ctypes.POINTER(GsOpts)], None),
    "gs_plan_create_from_mtx": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gs_plan_create_from_coo": ([ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p, f32p,
                                 ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gs_set_config_int": ([ctypes.c_char_p, ctypes.c_longlong], ctypes.c_int),
    "gs_get_config_int": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong)], ctypes.c_int),
    "gs_plan_add_operator": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int],
                             ctypes.c_int),
    "gs_plan_run_pipeline": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int],
                             ctypes.c_int),
    "gs_plan_add_operator_sub": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong),
                                  ctypes.c_int], ctypes.c_int),
    "gs_plan_run_pipeline_sub": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int], ctypes.c_int),
    "gs_plan_sub_matrices": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
    "gs_plan_compile": ([ctypes.c_void_p], ctypes.c_int),
    "gs_plan_generate_program": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int],
                                 ctypes.c_int),
    "gs_plan_upload": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "gs_plan_add_replica": ([ctypes.c_void_p], ctypes.c_int),
    "gs_spmm": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "gs_spmm_replica": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                         ctypes.c_void_p], ctypes.c_int),
    "gs_spmm_batch": ([ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p),
                       ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "gs_spmm_rotate": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "gs_batch_launches": ([ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
    "gs_plan_device_status": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "gs_plan_info_get": ([ctypes.c_void_p, ctypes.POINTER(GsPlanInfo)], ctypes.c_int),
    "gs_plan_array_count": ([ctypes.c_void_p], ctypes.c_int),
    "gs_plan_array_key": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "gs_plan_array_len": ([ctypes.c_void_p, ctypes.c_char_p], ctypes.c_longlong),
    "gs_plan_array_is_float": ([ctypes.c_void_p, ctypes.c_char_p], ctypes.c_int),
    "gs_plan_array_read_u64": ([ctypes.c_void_p, ctypes.c_char_p, u64p, ctypes.c_uint64], ctypes.c_int),
    "gs_plan_array_read_f64": ([ctypes.c_void_p, ctypes.c_char_p, f64p, ctypes.c_uint64], ctypes.c_int),
    "gs_plan_log": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "gs_plan_save": ([ctypes.c_void_p, ctypes.c_char_p], ctypes.c_int),
    "gs_plan_load": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gs_plan_index_compression": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                   ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "gs_index_compression_of_array": ([u64p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                       u64p, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "gs_debug_mfma_timeline": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64], ctypes.c_int),
    "gs_plan_from_mtx": ([ctypes.c_char_p, ctypes.POINTER(GsOpts), ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gs_plan_free": ([ctypes.c_void_p], None),
}

_lib = None


def load():
    """Loads libgeneralsparse.so.  torch (if importable) is imported first so that
    the process has one HIP runtime (torch's libamdhip64 shares the soname)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                           "(the GPU path has no fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


class GsError(RuntimeError):
    pass


GS_ERR_DEVICE = -4  # include/generalsparse.h: a kernel reported a fault in its device error word


def check(rc):
    if rc != 0:
        e = GsError(f"generalsparse error {rc}: {load().gs_last_error().decode()}")
        e.code = rc
        raise e
    return rc
