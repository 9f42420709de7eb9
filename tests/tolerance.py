"""Result tolerances of the GPU parity tests, in one place.

- The contract line (BASELINE.json north_star): fp32 1e-3, fp16 1e-1, relative to max(1, |ref|).
- The tight line for fp16 results of fp32-accumulating kernels: every family
  here accumulates in fp32 and rounds to fp16 once when it writes C, so the expected error is
  ~2^-11 |C| plus the fp32 accumulation error (far below 2^-11 at these row lengths); 2^-9
  relative to max(1, |ref|) is asserted as well.  It catches a dropped or doubled nonzero,
  which the contract line admits by the handful at C2 scale (|C| ~ 58, one term ~ 1.1).
- The exception: the bitmap family (k_bitmap_segment) adds the open-row partials of a plan
  without an fp32 workspace straight into fp16 C with atomics, as the reference's
  warp_segment kernel does (each add rounds to fp16), so it keeps the contract line only.
"""
import numpy as np

TOL = {"f32": 1e-3, "f16": 1e-1}
TIGHT_F16 = 2.0 ** -9
FP16_ATOMIC_KERNELS = ("k_bitmap_segment",)


def rel_err(C, ref):
    """max |C - ref| / max(1, |ref|) over all elements (numpy arrays)"""
    C = np.asarray(C, np.float64)
    ref = np.asarray(ref, np.float64)
    if C.size == 0:
        return 0.0
    return float((np.abs(C - ref) / np.maximum(1.0, np.abs(ref))).max())


def bound(dtype, kernel=None):
    """the bound a result of `kernel` (gs_plan_info.device_kernel) is held to"""
    if dtype == "f16" and not (kernel or "").startswith(FP16_ATOMIC_KERNELS):
        return TIGHT_F16
    return TOL[dtype]


def check(C, ref, dtype, kernel=None, what=""):
    err = rel_err(C, ref)
    b = bound(dtype, kernel)
    assert err <= b, f"{what} max rel err {err} > {b} ({dtype}, {kernel or 'fp32-accumulating'})"
    return err


def check_torch(C, ref, dtype, kernel=None, what=""):
    """the same on torch tensors (on the GPU): C, ref of one shape"""
    err = ((C.float() - ref.float()).abs() / ref.float().abs().clamp(min=1.0)).max().item()
    b = bound(dtype, kernel)
    assert err <= b, f"{what} max rel err {err} > {b} ({dtype}, {kernel or 'fp32-accumulating'})"
    return err
