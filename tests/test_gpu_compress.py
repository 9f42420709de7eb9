"""§8f rank 1 on the device: model-driven index compression consumed by the gather
kernels.

With MODEL_DRIVEN_COMPRESS the upload replaces every index array a gather kernel reads
(first_nz / first_row / first_BMW / the sort order) by the exact formula
index_compress.cc found -- the reference prints the same formulas into its generated
kernels (code_generator.cc:2618-3063) -- and the kernel evaluates it (gsk::idx_at).  The
product is checked here three ways on the same seeded inputs:
- bit-identical C with compression on and off (same kernel, same summation order) for
  the families without atomics; the bitmap / row-chunk families add rows shared between
  BMTs with fp32 atomics, whose order varies run to run: those agree to 1e-5,
- against the oracle (tolerances of north_star: fp32 1e-3, fp16 1e-1),
- the device bytes of A drop by exactly the bytes the formulas replace, and the
  fixed-blocking arrays (BMTB/BMW row starts, 32-nnz BMT starts) are formulas."""
import numpy as np
import pytest

import oracle_ffi as ofi

torch = pytest.importorskip("torch")
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
from tolerance import bound  # noqa: E402  (contract line + the tight fp16 line, tests/tolerance.py)

# (pipeline, p0, p1, arrays that must become formulas on the 400-row case)
PIPES = [("thread_total", 4, 1, 0), ("warp_total", 0, 1, 1), ("block_total", 0, 1, 1), ("block_total", 20, 1, 1),
         ("thread_bit_map", 4, 1, 2), ("warp_segment", 4, 1, 2), ("tblock_warp_total", 4, 1, 2),
         ("balanced_warp_total", 256, 1, 1), ("tblock_thread_total", 16, 1, 0)]
COL_PIPES = [("warp_bit_map", 4, 1, 0), ("tblock_bit_map", 4, 1, 0)]
ATOMIC = ("thread_bit_map", "warp_segment", "warp_bit_map", "tblock_bit_map")


@pytest.fixture
def gather_only():
    """the formulas are consumed by the gather families: keep fp16 BMTB plans off the
    matrix-core and LDS-stage kernels for this test"""
    gsa.set_config("MFMA_TILES", 0)
    gsa.set_config("LDS_STAGE_B", 0)
    yield
    gsa.set_config("MFMA_TILES", 1)
    gsa.set_config("LDS_STAGE_B", 1)
    gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)


def run(M, K, row, col, val, pipe, p0, p1, N, dtype, B, compress):
    gsa.set_config("MODEL_DRIVEN_COMPRESS", 1 if compress else 0)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile().upload(dtype, 0)
    gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)
    C = plan.spmm(torch.from_numpy(B).to(DEV))
    torch.cuda.synchronize()
    info = plan.info()
    plan.free()
    return C.float().cpu().numpy(), info


def cases(col_direction):
    if col_direction:
        yield 300, 2000, *ds.random_rows(300, 2000, 150.0, seed=11, empty_frac=0.1)
        r, c, v = ds.two_four(96, 512, 30)
        yield 96, 512, r, c, v
    else:
        yield 400, 300, *ds.random_rows(400, 300, 12.0, seed=1, empty_frac=0.1)
        yield 1024, 1024, *ds.rmat(1024, 20000, seed=2)
        rows = np.concatenate([np.zeros(3000, np.uint64), np.arange(1, 50, dtype=np.uint64)])
        cols = np.concatenate([np.arange(3000, dtype=np.uint64), np.arange(1, 50, dtype=np.uint64) % 3000])
        yield 60, 3000, rows, cols, np.linspace(-1, 1, len(rows)).astype(np.float32)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 32, 13])
@pytest.mark.parametrize("pipe", PIPES + COL_PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_formulas_on_device_match(pipe, N, dtype, gather_only):
    name, p0, p1, want = pipe
    col_dir = (name, p0, p1, want) in COL_PIPES
    npdt = np.float16 if dtype == "f16" else np.float32
    for i, (M, K, row, col, val) in enumerate(cases(col_dir)):
        if name == "balanced_warp_total" and M == 60:
            continue  # trailing empty rows: the reference splitter asserts (tested on CPU)
        if col_dir and dtype == "f16" and N == 32 and M == 96:
            continue  # 2:4 panels on the sparse matrix cores (no index arrays)
        B = np.random.default_rng(i).uniform(-1, 1, (K, N)).astype(npdt)
        C0, i0 = run(M, K, row, col, val, name, p0, p1, N, dtype, B, False)
        C1, i1 = run(M, K, row, col, val, name, p0, p1, N, dtype, B, True)
        assert i0["device_kernel"] == i1["device_kernel"]
        assert i0["index_formulas"] == 0 and i0["index_bytes_saved"] == 0
        assert i1["device_bytes_A"] + i1["index_bytes_saved"] == i0["device_bytes_A"], (i0, i1)
        if i == 0:
            assert i1["index_formulas"] >= want, (name, i1)
        if name in ATOMIC:
            np.testing.assert_allclose(C1, C0, rtol=1e-5, atol=1e-5)
        else:
            np.testing.assert_array_equal(C1, C0)
        v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        err = np.abs(C1 - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= bound(dtype, i1["device_kernel"]), (name, M, i1["device_kernel"], err.max())


def test_fixed_blocking_arrays_leave_hbm(gather_only):
    """tblock_warp_total(4, 1) on 4000 rows: the BMW row starts (4001 u32) and the BMTB ->
    BMW map (1001 u32) are linear, so 20,008 bytes of index arrays are not uploaded"""
    M, K, N = 4000, 3000, 32
    row, col, val = ds.random_rows(M, K, 12.0, seed=1)
    B = np.random.default_rng(0).uniform(-1, 1, (K, N)).astype(np.float32)
    C0, i0 = run(M, K, row, col, val, "tblock_warp_total", 4, 1, N, "f32", B, False)
    C1, i1 = run(M, K, row, col, val, "tblock_warp_total", 4, 1, N, "f32", B, True)
    assert i1["index_formulas"] == 2 and i1["index_bytes_saved"] == (4001 + 1001) * 4
    np.testing.assert_array_equal(C1, C0)
