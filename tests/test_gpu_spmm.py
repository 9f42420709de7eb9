"""GPU parity (run on the MI355X box with -m gpu): every kernel family, through
the C ABI, against the oracle on the same seeded inputs.

Tolerances (BASELINE.json north_star): fp32 1e-3, fp16 1e-1, relative to
max(1, |ref|).  The reference's own known answer (all-ones A and B =>
C[i][j] = nnz(row i), exact) is checked bit-exactly.  At full C2 size the
result is checked against a plain PyTorch fp32 dense matmul of the same fp16
inputs."""
import numpy as np
import pytest

import oracle_ffi as ofi

torch = pytest.importorskip("torch")
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402
from build_flags import need_experiments  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
PIPES = [("thread_total", 4, 1), ("thread_total", 8, 1), ("warp_total", 0, 1), ("block_total", 0, 1),
         ("block_total", 20, 1),
         ("thread_bit_map", 4, 1), ("warp_segment", 4, 1), ("tblock_warp_total", 4, 1),
         ("tblock_warp_total", 16, 1), ("tblock_warp_total", 32, 8), ("tblock_warp_total", 64, 16),
         ("balanced_warp_total", 256, 1),
         ("merge_path", 1024, 1), ("merge_path", 64, 1), ("merge_path", 7, 3), ("merge_path", 4096, 2),
         ("balanced_block_total", 512, 1), ("balanced_thread_total", 64, 1),
         ("tblock_thread_total", 16, 1), ("tblock_thread_total", 20, 3), ("tblock_warp_thread_total", 16, 2)]
BALANCED = ("balanced_warp_total", "balanced_block_total", "balanced_thread_total")
from tolerance import TOL, bound  # noqa: E402  (contract line + the tight fp16 line, tests/tolerance.py)


def run(M, K, row, col, val, pipeline, p0, p1, N, dtype, B=None, seed=0):
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipeline, N, p0, p1).compile().upload(dtype, 0)
    npdt = np.float16 if dtype == "f16" else np.float32
    if B is None:
        B = np.random.default_rng(seed).uniform(-1, 1, (K, N)).astype(npdt)
    Bt = torch.from_numpy(B).to(DEV)
    C = plan.spmm(Bt)
    torch.cuda.synchronize()
    return plan, C.float().cpu().numpy(), B


def check(C, ref, dtype, plan=None):
    """the contract tolerance, and 2^-9 for the fp16 results of fp32-accumulating kernels
    (every kernel but the bitmap family's fp16 atomics, tests/tolerance.py)"""
    kernel = plan.info()["device_kernel"] if plan is not None else None
    err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
    b = bound(dtype, kernel)
    assert err.max() <= b, f"max rel err {err.max()} > {b} ({kernel})"


def coo_cases():
    yield "random", 300, 200, *ds.random_rows(300, 200, 12.0, seed=1, empty_frac=0.15)
    yield "powerlaw", 1024, 1024, *ds.rmat(1024, 20000, seed=2)
    r, c, v = ds.pruned_weight(256, 512, 0.7, 13)
    yield "pruned", 256, 512, r, c, v
    # ragged: one very long row among short ones, trailing empty rows
    rows = np.concatenate([np.zeros(3000, np.uint64), np.arange(1, 50, dtype=np.uint64)])
    cols = np.concatenate([np.arange(3000, dtype=np.uint64), np.arange(1, 50, dtype=np.uint64) % 3000])
    yield "ragged", 60, 3000, rows, cols, np.linspace(-1, 1, len(rows)).astype(np.float32)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 32, 13])
@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_spmm_matches_oracle(pipe, N, dtype):
    name, p0, p1 = pipe
    for case, M, K, row, col, val in coo_cases():
        if name in BALANCED and case == "ragged":
            continue  # trailing empty rows: the reference splitter asserts (tested on CPU)
        plan, C, B = run(M, K, row, col, val, name, p0, p1, N, dtype)
        v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        check(C, ref, dtype, plan)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_known_answer_all_ones(pipe, dtype):
    name, p0, p1 = pipe
    M, K, N = 400, 300, 32
    row, col, _ = ds.random_rows(M, K, 20.0, seed=7, empty_frac=0.1)
    ones = np.ones(len(row), np.float32)
    npdt = np.float16 if dtype == "f16" else np.float32
    _, C, _ = run(M, K, row, col, ones, name, p0, p1, N, dtype, B=np.ones((K, N), npdt))
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 32])
@pytest.mark.parametrize("pipe", [("block_total", 2500, 1), ("balanced_block_total", 2048, 1),
                                  ("block_total", 1024, 1)], ids=lambda p: f"{p[0]}-{p[1]}")
def test_block_rows_short_and_long_rows(pipe, N, dtype):
    """k_block_rows: slot-per-row walks of short rows, the workgroup-wide reduction of
    rows over kBrSolo nonzeros, and BMTBs of more than one 1024-row window"""
    name, p0, p1 = pipe
    M = K = 3000
    row, col, val = ds.rmat(M, 24000, seed=5)
    # a few long rows (> 64 nnz) in the middle of short ones
    extra_r = np.repeat(np.array([17, 1100, 2999], np.uint64), 300)
    extra_c = np.tile(np.arange(300, dtype=np.uint64) * 9, 3)
    keep = ~np.isin(row, [17, 1100, 2999])
    row = np.concatenate([row[keep], extra_r])
    col = np.concatenate([col[keep], extra_c])
    val = np.concatenate([val[keep], np.linspace(-1, 1, len(extra_r)).astype(np.float32)])
    o = np.lexsort((col, row))
    row, col, val = row[o], col[o], val[o]
    plan, C, B = run(M, K, row, col, val, name, p0, p1, N, dtype)
    assert plan.info()["device_kernel"] == "k_block_rows"
    v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
    check(C, ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64"), dtype, plan)


# col-direction pipelines (K5 warp_bit_map / K7 tblock_bit_map): BMTs are 64-nnz
# chunks of one row, so the cases need rows long enough for the padding rule
COL_PIPES = [("warp_bit_map", 4, 1), ("tblock_bit_map", 4, 1), ("warp_bit_map_interleaved", 4, 1),
             ("tblock_bit_map_interleaved", 4, 1)]


def col_cases():
    yield "long", 300, 2000, *ds.random_rows(300, 2000, 150.0, seed=11, empty_frac=0.1)
    r, c, v = ds.pruned_weight(256, 512, 0.7, 13)
    yield "pruned", 256, 512, r, c, v
    r, c, v = ds.two_four(96, 512, 30)
    yield "2:4", 96, 512, r, c, v
    # rows of 47 BMTs straddle several waves' ranges (fp32 workspace + finalize path)
    rows = np.concatenate([np.zeros(3000, np.uint64), np.repeat(np.arange(1, 40, dtype=np.uint64), 70)])
    cols = np.concatenate([np.arange(3000, dtype=np.uint64), np.tile(np.arange(70, dtype=np.uint64) * 7, 39)])
    yield "ragged", 45, 3000, rows, cols, np.linspace(-1, 1, len(rows)).astype(np.float32)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 32, 13, 128])
@pytest.mark.parametrize("pipe", COL_PIPES, ids=lambda p: p[0])
def test_col_direction_matches_oracle(pipe, N, dtype):
    name, p0, p1 = pipe
    for case, M, K, row, col, val in col_cases():
        plan, C, B = run(M, K, row, col, val, name, p0, p1, N, dtype)
        assert plan.info()["kernel_name"].startswith("k_row_chunks"), plan.info()["kernel_name"]
        # 2:4 rows of an fp16 plan at N = 32/64/128 run on the sparse matrix cores
        # (tests/test_gpu_nm.py); everything else on the row-chunk kernel
        nm = case == "2:4" and dtype == "f16" and N in (8, 16, 32, 64, 128) and "interleaved" not in name
        assert plan.info()["lds_stage"] == (3 if nm else 0), (case, plan.info())
        v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        check(C, ref, dtype, plan)
        # the workspace is re-zeroed by the finalize pass: a second launch agrees
        C2 = plan.spmm(torch.from_numpy(B).to(DEV)).float().cpu().numpy()
        check(C2, ref, dtype, plan)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", COL_PIPES, ids=lambda p: p[0])
def test_col_direction_known_answer(pipe, dtype):
    name, p0, p1 = pipe
    M, K, N = 200, 1500, 32
    row, col, _ = ds.random_rows(M, K, 300.0, seed=9, empty_frac=0.1)
    npdt = np.float16 if dtype == "f16" else np.float32
    _, C, _ = run(M, K, row, col, np.ones(len(row), np.float32), name, p0, p1, N, dtype, B=np.ones((K, N), npdt))
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))


def test_col_direction_wider_B_is_refused():
    row, col, val = ds.random_rows(64, 600, 100.0, seed=2)
    plan = gsa.Plan.from_coo(64, 600, row, col, val).run_pipeline("warp_bit_map", 32, 4, 1).compile().upload("f16", 0)
    with pytest.raises(gsa.GsError):
        plan.spmm(torch.zeros((600, 64), device=DEV, dtype=torch.float16))


def test_replicas_and_stream():
    M, K, N = 500, 400, 32
    row, col, val = ds.random_rows(M, K, 15.0, seed=3)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("tblock_warp_total", N, 4, 1).compile().upload("f16", 0)
    plan.add_replica()
    plan.add_replica()
    B = torch.rand((K, N), device=DEV, dtype=torch.float16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        outs = [plan.spmm(B, replica=i) for i in range(3)]
    s.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    assert plan.info()["replicas"] == 3


def test_operands_are_checked_before_any_launch():
    """a C the kernels would write out of bounds (short, strided, wrong dtype) and a B of the
    wrong shape are refused by spmm / rotation / Batch; C is left untouched; a checked
    rotation then runs the same SpMM as spmm"""
    M, K, N = 300, 200, 16
    row, col, val = ds.random_rows(M, K, 12.0, seed=5)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, 40, 1).compile().upload("f16", 0)
    B = torch.rand((K, N), device=DEV, dtype=torch.float16)
    good = torch.empty((M, N), device=DEV, dtype=torch.float16)
    bad_C = [torch.zeros((M - 1, N), device=DEV, dtype=torch.float16),
             torch.zeros((N, M), device=DEV, dtype=torch.float16).t(),
             torch.zeros((M, N), device=DEV, dtype=torch.float32),
             torch.zeros((M, N + 8), device=DEV, dtype=torch.float16)]
    for C in bad_C:
        with pytest.raises((ValueError, TypeError)):
            plan.spmm(B, C=C)
        with pytest.raises(ValueError):
            plan.rotation([B], [C])
        with pytest.raises(ValueError):
            gsa.Batch([(plan, 0, B, C)], N)
        assert not C.any()
    with pytest.raises(ValueError):
        plan.spmm(torch.rand((K + 1, N), device=DEV, dtype=torch.float16))
    with pytest.raises(ValueError):
        plan.rotation([B, B], [good])
    with pytest.raises(ValueError):
        plan.rotation([B, torch.rand((K, 2 * N), device=DEV, dtype=torch.float16)], [good, good.clone()])
    ref = plan.spmm(B)
    plan.rotation([B], [good]).run(3, 0)
    torch.cuda.synchronize()
    assert torch.equal(good, ref)


def test_c2_full_size_against_torch():
    """BASELINE configs[1] shape: OPT-13B q_proj stand-in 5120x5120, 70% pruned, fp16, N=32"""
    M = K = 5120
    N = 32
    row, col, val = ds.pruned_weight(M, K, 0.7, 13)
    assert len(row) == 7864320
    A = torch.zeros((M, K), dtype=torch.float32)
    A[torch.from_numpy(row.astype(np.int64)), torch.from_numpy(col.astype(np.int64))] = \
        torch.from_numpy(val).half().float()
    A = A.to(DEV)
    B = torch.randn((K, N), device=DEV, dtype=torch.float16)
    ref = A @ B.float()
    for name, p0, p1 in (("tblock_warp_total", 20, 2), ("tblock_warp_total", 4, 1), ("warp_segment", 4, 1),
                         ("thread_total", 4, 1), ("block_total", 0, 1)):
        plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile().upload("f16", 0)
        C = plan.spmm(B).float()
        torch.cuda.synchronize()
        err = ((C - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
        assert err <= bound("f16", plan.info()["device_kernel"]), (name, plan.info()["device_kernel"], err)
        # linearity: A(2B) = 2 AB.  Deterministic families (no atomics) are exact;
        # the bitmap family adds open row partials into fp16 C with atomics, as the
        # reference's warp_segment kernel does: each add rounds to fp16 (ulp 2^-5 at
        # the partials' magnitude ~40), so a cancelling row of |C| ~ 1 can differ by
        # a few ulps between the two runs
        C2 = plan.spmm((B * 2)).float()
        lin = ((C2 - 2 * C).abs() / (2 * C).abs().clamp(min=1.0)).max().item()
        if name == "warp_segment":
            assert lin <= 2.5e-1, (name, lin)
        else:
            assert lin == 0.0, (name, lin)


def test_rocsparse_comparator_agrees():
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(gsa.__file__), "librocsparse_cmp.so"))
    M, K, N = 512, 384, 32
    row, col, val = ds.random_rows(M, K, 16.0, seed=4)
    rp = np.zeros(M + 1, np.int32)
    np.add.at(rp, row.astype(np.int64) + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    c32 = col.astype(np.int32)
    v = val.astype(np.float32)
    out = np.zeros((M, N), np.float32)
    ms = ctypes.c_double()
    rc = lib.rs_spmm_bench(M, K, len(v), rp.ctypes.data_as(ctypes.c_void_p), c32.ctypes.data_as(ctypes.c_void_p),
                           v.ctypes.data_as(ctypes.c_void_p), N, 0, 0, 1, 2, 1, ctypes.byref(ms),
                           out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    B = np.array([(i * 2654435761) % 1000 / 1000.0 - 0.5 for i in range(K * N)],
                 np.float32).reshape(K, N)
    ref = ofi.spmm_ref(M, N, row, col, v, B, "f64")
    check(out, ref, "f32")


# ---------------------------------------------------------------- LDS-stationary B
# tblock_warp_total(p0 rows per BMTB, p1 rows per BMW) uploads the chunk-major tile
# layout and runs k_lds_rows when dense width N makes whole 16-B B rows.
LDS_PIPES = [(20, 2), (16, 2), (64, 4), (32, 4), (48, 3)]


def lds_cases():
    yield from coo_cases()
    # many column chunks: K far above one LDS chunk of B
    yield "wide", 300, 40000, *ds.random_rows(300, 40000, 300.0, seed=5, empty_frac=0.05)


@pytest.fixture
def no_mfma():
    gsa.set_config("MFMA_TILES", 0)
    yield
    gsa.set_config("MFMA_TILES", 1)


@pytest.mark.parametrize("dtype,N", [("f16", 8), ("f16", 32), ("f16", 64), ("f32", 4), ("f32", 32)])
@pytest.mark.parametrize("pipe", LDS_PIPES, ids=lambda p: f"{p[0]}x{p[1]}")
def test_lds_stage_matches_oracle(pipe, dtype, N, no_mfma):
    p0, p1 = pipe
    for case, M, K, row, col, val in lds_cases():
        plan, C, B = run(M, K, row, col, val, "tblock_warp_total", p0, p1, N, dtype)
        info = plan.info()
        assert info["lds_stage"] == 1 and info["lds_n"] == N, (case, info)
        v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        check(C, ref, dtype, plan)
        # a different dense width than the plan's falls back to the gather kernel
        N2 = N + 1
        B2 = np.random.default_rng(1).uniform(-1, 1, (K, N2)).astype(B.dtype)
        C2 = plan.spmm(torch.from_numpy(B2).to(DEV)).float().cpu().numpy()
        ref2 = ofi.spmm_ref(M, N2, row, col, v, B2.astype(np.float32), "f64")
        check(C2, ref2, dtype, plan)
        plan.free()


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("ksplit", [0, 2, 3])
def test_lds_stage_k_split(dtype, ksplit, no_mfma):
    """k_lds_rows with its BMTBs' K split over workgroups (LDS_KSPLIT; 0 = the upload's rule:
    plans of under 128 BMTBs split until ~256 workgroups): the fp32 slab combine against the
    oracle, a relaunch into a NaN-filled C bit for bit (the arrival counters re-arm), and the
    unsplit plan within the tolerance"""
    M, K = 600, 30000
    row, col, val = ds.random_rows(M, K, 400.0, seed=21, empty_frac=0.05)
    N = 32
    gsa.set_config("LDS_KSPLIT", ksplit)
    try:
        plan, C, B = run(M, K, row, col, val, "tblock_warp_total", 20, 2, N, dtype)
    finally:
        gsa.set_config("LDS_KSPLIT", 0)
    info = plan.info()
    assert info["device_kernel"].startswith("k_lds_rows") and info["ksplit"] > 1, info
    if ksplit:
        assert info["ksplit"] == ksplit, info
    v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
    check(C, ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64"), dtype, plan)
    Bt = torch.from_numpy(B).to(DEV)
    C2 = torch.full((M, N), float("nan"), device=DEV, dtype=Bt.dtype)
    plan.spmm(Bt, C=C2)
    plan.spmm(Bt, C=C2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(C2.float().cpu().numpy(), C)
    plan.free()


@pytest.mark.parametrize("ksplit", [1, 0, 3])
def test_lds_stage_dma_fp32(ksplit, no_mfma):
    """LDS_DMA (fp32, N = 32): k_lds_rows_dma stages every chunk's B rows and A segment by
    LDS-DMA into two buffers (chunk j+1 lands while chunk j is computed): against the oracle on
    every LDS case (including 40,000 columns: many chunks), with and without the K split, and a
    relaunch into NaN-filled C bit for bit"""
    assert gsa.get_config("LDS_DMA") == 1  # the default
    gsa.set_config("LDS_KSPLIT", ksplit)
    try:
        for case, M, K, row, col, val in lds_cases():
            for p0, p1 in ((20, 2), (16, 4), (64, 4)):
                plan, C, B = run(M, K, row, col, val, "tblock_warp_total", p0, p1, 32, "f32")
                info = plan.info()
                assert info["device_kernel"] == "k_lds_rows_dma", (case, info)
                check(C, ofi.spmm_ref(M, 32, row, col, val, B, "f64"), "f32", plan)
                Bt = torch.from_numpy(B).to(DEV)
                C2 = torch.full((M, 32), float("nan"), device=DEV)
                plan.spmm(Bt, C=C2)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(C2.cpu().numpy(), C)
                plan.free()
    finally:
        gsa.set_config("LDS_KSPLIT", 0)


@pytest.mark.parametrize("ksplit", [1, 0, 3])
def test_lds_stage_rowslot_fp32(ksplit, no_mfma):
    """BMWs of 5..8 rows at fp32, N = 32: k_lds_rows_rs (one row per slot, rows' entries in the
    slot-parity order) against the oracle on every LDS case, with and without the K split, a
    relaunch into NaN-filled C bit for bit, and the all-ones known answer exactly
    (code_generator.cc:633-637: every C[i][j] is row i's nonzero count)"""
    gsa.set_config("LDS_KSPLIT", ksplit)
    try:
        for case, M, K, row, col, val in lds_cases():
            for p0, p1 in ((64, 8), (40, 5), (48, 6), (16, 8)):
                plan, C, B = run(M, K, row, col, val, "tblock_warp_total", p0, p1, 32, "f32")
                info = plan.info()
                assert info["device_kernel"] == "k_lds_rows_rs", (case, p0, p1, info)
                check(C, ofi.spmm_ref(M, 32, row, col, val, B, "f64"), "f32", plan)
                Bt = torch.from_numpy(B).to(DEV)
                C2 = torch.full((M, 32), float("nan"), device=DEV)
                plan.spmm(Bt, C=C2)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(C2.cpu().numpy(), C)
                plan.free()
            ones, C1, _ = run(M, K, row, col, np.ones(len(row), np.float32), "tblock_warp_total", 64, 8, 32, "f32",
                              B=np.ones((K, 32), np.float32))
            assert ones.info()["device_kernel"] == "k_lds_rows_rs"
            nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
            np.testing.assert_array_equal(C1, np.repeat(nnz_row[:, None], 32, axis=1))
            ones.free()
    finally:
        gsa.set_config("LDS_KSPLIT", 0)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_lds_stage_known_answer(dtype, no_mfma):
    M, K, N = 700, 9000, 32
    row, col, _ = ds.random_rows(M, K, 60.0, seed=8, empty_frac=0.1)
    npdt = np.float16 if dtype == "f16" else np.float32
    plan, C, _ = run(M, K, row, col, np.ones(len(row), np.float32), "tblock_warp_total", 20, 2, N, dtype,
                     B=np.ones((K, N), npdt))
    assert plan.info()["lds_stage"] == 1
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))


def test_lds_stage_off_and_unfit_plans_use_gather_kernel(no_mfma):
    M, K, N = 300, 500, 32
    row, col, val = ds.random_rows(M, K, 10.0, seed=9)
    try:
        gsa.set_config("LDS_STAGE_B", 0)
        plan, C0, B = run(M, K, row, col, val, "tblock_warp_total", 20, 2, N, "f16")
        assert plan.info()["lds_stage"] == 0
    finally:
        gsa.set_config("LDS_STAGE_B", 1)
    plan1, C1, _ = run(M, K, row, col, val, "tblock_warp_total", 20, 2, N, "f16", B=B)
    assert plan1.info()["lds_stage"] == 1
    check(C1, C0, "f16")
    # 64 one-row BMWs per BMTB exceed the 16-wave workgroup, and 4-row BMTBs are
    # faster gathered: gather kernel
    for p0, p1 in ((64, 1), (4, 1)):
        plan2, C2, _ = run(M, K, row, col, val, "tblock_warp_total", p0, p1, N, "f16", B=B)
        assert plan2.info()["lds_stage"] == 0
        check(C2, C0, "f16")


# ---------------------------------------------------------------- matrix-core row blocks
# fp16 plans with BMTB row blocks run k_mfma_rows when the blocks are dense enough
# (MFMA_MAX_FILL); the tests raise the fill limit so sparse cases exercise it too.
MFMA_PIPES = [("tblock_warp_total", 20, 2), ("block_total", 16, 1), ("block_total", 20, 1),
              ("block_total", 33, 1), ("block_total", 64, 1), ("block_total", 7, 1)]


def mfma_cases():
    yield from coo_cases()
    r, c, v = ds.pruned_weight(1000, 3000, 0.8, 21)
    yield "pruned_ragged_M", 1000, 3000, r, c, v
    r, c, v = ds.pruned_weight(300, 4100, 0.5, 22)  # K not a multiple of the chunk or of 32
    yield "pruned_odd_K", 300, 4100, r, c, v
    keep = (r % 7) != 3  # empty rows inside row blocks
    yield "pruned_empty_rows", 300, 4100, r[keep], c[keep], v[keep]


@pytest.fixture
def mfma_everywhere():
    gsa.set_config("MFMA_MAX_FILL", 1 << 30)
    yield
    gsa.set_config("MFMA_MAX_FILL", 16)
    gsa.set_config("MFMA_GLDS", 1)
    gsa.set_config("MFMA_KS", 1)


@pytest.mark.parametrize("glds", [1, 0])  # B rows by LDS-DMA (default) / through registers
@pytest.mark.parametrize("N", [8, 16, 32, 64])
@pytest.mark.parametrize("pipe", MFMA_PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_mfma_rows_match_oracle(pipe, N, glds, mfma_everywhere):
    name, p0, p1 = pipe
    gsa.set_config("MFMA_GLDS", glds)
    # every case must be right whichever kernel the upload picked; the matrix
    # cores must have taken at least one case (33..64-row blocks at N=64 never
    # fit LDS twice over, and 50%-dense chunks of them exceed the stage buffers)
    used = []
    for case, M, K, row, col, val in mfma_cases():
        plan, C, B = run(M, K, row, col, val, name, p0, p1, N, "f16")
        used.append(plan.info()["device_kernel"])
        v = val.astype(np.float16).astype(np.float32)
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        check(C, ref, "f16")
        plan.free()
    if not (p0 > 32 and N == 64):
        assert any(k in ("k_mfma_rows", "k_mfma_ks") for k in used), used


# K-split matrix-core kernel (k_mfma_ks): row blocks of >= KS_MIN_ROWS rows, K ranges per
# row block (KS_SPLIT; 0 = enough workgroups for the CUs), slabs combined by the last arriver
KS_PIPES = [("block_total", 40, 1), ("block_total", 48, 1), ("block_total", 64, 1), ("block_total", 80, 1),
            ("tblock_warp_total", 80, 2)]


@pytest.mark.parametrize("split", [0, 1, 3])
@pytest.mark.parametrize("N", [8, 16, 24, 32, 64, 128])
@pytest.mark.parametrize("pipe", KS_PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_mfma_ks_matches_oracle(pipe, N, split, mfma_everywhere):
    name, p0, p1 = pipe
    gsa.set_config("KS_SPLIT", split)
    used = []
    try:
        for case, M, K, row, col, val in mfma_cases():
            plan, C, B = run(M, K, row, col, val, name, p0, p1, N, "f16")
            info = plan.info()
            used.append(info["device_kernel"])
            v = val.astype(np.float16).astype(np.float32)
            ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
            check(C, ref, "f16")
            if info["device_kernel"] == "k_mfma_ks":
                # deterministic whichever K range arrives last; arrival counters reset; replicas agree
                Bt = torch.from_numpy(B).to(DEV)
                np.testing.assert_array_equal(plan.spmm(Bt).float().cpu().numpy(), C)
                plan.add_replica()
                np.testing.assert_array_equal(plan.spmm(Bt, replica=1).float().cpu().numpy(), C)
            plan.free()
    finally:
        gsa.set_config("KS_SPLIT", 0)
    assert "k_mfma_ks" in used, used


@pytest.mark.parametrize("split", [0, 1, 3])
@pytest.mark.parametrize("N", [8, 24, 32])
@pytest.mark.parametrize("rows", [96, 112, 128])
def test_mfma_ks_tall_blocks_match_oracle(rows, N, split, mfma_everywhere):
    """96..128-row blocks (RT 6..8: whole CU rounds on the OPT-30B shapes) at N <= 32"""
    gsa.set_config("KS_SPLIT", split)
    used = []
    try:
        for case, M, K, row, col, val in mfma_cases():
            plan, C, B = run(M, K, row, col, val, "block_total", rows, 1, N, "f16")
            info = plan.info()
            used.append(info["device_kernel"])
            ref = ofi.spmm_ref(M, N, row, col, val.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
            check(C, ref, "f16")
            if info["device_kernel"] == "k_mfma_ks":
                np.testing.assert_array_equal(plan.spmm(torch.from_numpy(B).to(DEV)).float().cpu().numpy(), C)
            plan.free()
    finally:
        gsa.set_config("KS_SPLIT", 0)
    assert "k_mfma_ks" in used, used


@pytest.mark.parametrize("split", [1, 2, 4])
@pytest.mark.parametrize("rows", [40, 64, 80])
def test_mfma_ks_overlapped_lds_layout(rows, split, mfma_everywhere):
    """KS_APART = 0: the partial tiles reuse the stage LDS after the loop barrier (more
    workgroups per CU); same sums in the same order as the apart layout: bit-identical C"""
    need_experiments()
    N = 32
    r, c, v = ds.pruned_weight(640, 2048, 0.7, 6)
    B = torch.from_numpy(np.random.default_rng(2).uniform(-1, 1, (2048, N)).astype(np.float16)).to(DEV)
    outs = []
    gsa.set_config("KS_SPLIT", split)
    try:
        for ap in (1, 0):
            gsa.set_config("KS_APART", ap)
            plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", N, rows, 1).compile().upload("f16", 0)
            info = plan.info()
            assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == split, info
            outs.append((plan.spmm(B).float().cpu().numpy(), info["lds_bytes"]))
            plan.spmm(B)
            plan.device_status()
            plan.free()
    finally:
        gsa.set_config("KS_APART", 1)
        gsa.set_config("KS_SPLIT", 0)
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[1][1] <= outs[0][1]
    check(outs[1][0], ofi.spmm_ref(640, N, r, c, v.astype(np.float16).astype(np.float32),
                                   B.cpu().numpy().astype(np.float32), "f64"), "f16")


@pytest.mark.parametrize("split", [0, 1, 3])
@pytest.mark.parametrize("rows", [40, 56, 80, 112, 128])
def test_mfma_ks_pos8_layout_is_exact(rows, split, mfma_everywhere):
    """KS_POS8: 8-bit entry positions in 8 x 16 segments (3 B per nonzero) build the same wave
    images as the u16 positions, so C is bit-identical (and matches the oracle), single and
    grouped launches alike"""
    need_experiments()
    N = 32
    cases = [ds.pruned_weight(640, 2048, 0.7, 8), ds.random_rows(640, 2048, 400.0, seed=3, empty_frac=0.2)]
    gsa.set_config("KS_SPLIT", split)
    try:
        for r, c, v in cases:
            B = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, (2048, N)).astype(np.float16)).to(DEV)
            outs, plans = [], []
            for p8 in (0, 1):
                gsa.set_config("KS_POS8", p8)
                plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", N, rows, 1).compile().upload("f16", 0)
                info = plan.info()
                assert info["device_kernel"] == "k_mfma_ks", info
                outs.append((plan.spmm(B).float().cpu().numpy(), info["tile_bytes"]))
                plans.append(plan)
            np.testing.assert_array_equal(outs[0][0], outs[1][0])
            assert outs[1][1] < outs[0][1], (outs[1][1], outs[0][1])
            check(outs[1][0], ofi.spmm_ref(640, N, r, c, v.astype(np.float16).astype(np.float32),
                                           B.cpu().numpy().astype(np.float32), "f64"), "f16")
            # grouped: two P8 entries in one k_mfma_ks_group launch
            plans[1].add_replica()
            Cs = [torch.full((640, N), float("nan"), device=DEV, dtype=torch.float16) for _ in range(2)]
            bat = gsa.Batch([(plans[1], 0, B, Cs[0]), (plans[1], 1, B, Cs[1])], N)
            assert bat.launches() == [2]
            bat.run(torch.cuda.current_stream().cuda_stream)
            for cc in Cs:
                np.testing.assert_array_equal(cc.float().cpu().numpy(), outs[0][0])
            for p in plans:
                p.device_status()
                p.free()
    finally:
        gsa.set_config("KS_POS8", 0)
        gsa.set_config("KS_SPLIT", 0)


@pytest.mark.parametrize("split", [0, 1, 3])
@pytest.mark.parametrize("rows,N", [(40, 32), (80, 32), (112, 32), (40, 128), (48, 128)])
def test_mfma_ks_nontemporal_loads_bit_identical(rows, N, split, mfma_everywhere):
    """KS_NT (a plan-search variant of the default build): A's groups by non-temporal loads --
    the same kernel arithmetic, so C is the KS_NT=0 kernel's bit for bit (and the oracle's),
    single and grouped launches alike; a group does not mix the two forms"""
    cases = [ds.pruned_weight(640, 2048, 0.7, 9), ds.random_rows(640, 2048, 400.0, seed=4, empty_frac=0.2)]
    gsa.set_config("KS_SPLIT", split)
    try:
        for r, c, v in cases:
            B = torch.from_numpy(np.random.default_rng(6).uniform(-1, 1, (2048, N)).astype(np.float16)).to(DEV)
            outs, plans = [], []
            for nt in (0, 1):
                gsa.set_config("KS_NT", nt)
                plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", N, rows, 1).compile().upload("f16", 0)
                assert plan.info()["device_kernel"] == "k_mfma_ks", plan.info()
                outs.append(plan.spmm(B).float().cpu().numpy())
                plans.append(plan)
            gsa.set_config("KS_NT", 0)
            for o in outs[1:]:
                np.testing.assert_array_equal(outs[0], o)
            check(outs[1], ofi.spmm_ref(640, N, r, c, v.astype(np.float16).astype(np.float32),
                                        B.cpu().numpy().astype(np.float32), "f64"), "f16")
            if N != 32:  # grouped launches are built for N = 32
                for p in plans:
                    p.free()
                continue
            plans[1].add_replica()
            Cs = [torch.full((640, N), float("nan"), device=DEV, dtype=torch.float16) for _ in range(3)]
            bat = gsa.Batch([(plans[1], 0, B, Cs[0]), (plans[1], 1, B, Cs[1])], N)
            assert bat.launches() == [2]
            bat.run(torch.cuda.current_stream().cuda_stream)
            mixed = gsa.Batch([(plans[0], 0, B, Cs[2]), (plans[1], 0, B, Cs[0])], N)
            assert sorted(mixed.launches()) == [1, 1]
            mixed.run(torch.cuda.current_stream().cuda_stream)
            for cc in Cs:
                np.testing.assert_array_equal(cc.float().cpu().numpy(), outs[0])
            for p in plans:
                p.device_status()
                p.free()
    finally:
        gsa.set_config("KS_NT", 0)
        gsa.set_config("KS_SPLIT", 0)


@pytest.mark.parametrize("nt", [0, 1])
@pytest.mark.parametrize("rows,split", [(40, 0), (40, 2), (80, 4), (112, 1), (112, 4), (128, 3)])
def test_mfma_ks_head_steps_bit_identical(rows, split, nt, mfma_everywhere):
    """KS_HEAD (default 1): each wave's first k-steps at fixed, padded slots, loaded without their
    records -- the padding groups write zeros into the image's zero row, so C is the record-only
    layout's bit for bit (single and grouped launches, with and without KS_NT), and the oracle's"""
    N = 32
    cases = [ds.pruned_weight(640, 2048, 0.7, 10), ds.random_rows(640, 2048, 400.0, seed=5, empty_frac=0.2)]
    gsa.set_config("KS_SPLIT", split)
    gsa.set_config("KS_NT", nt)
    try:
        for r, c, v in cases:
            B = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, (2048, N)).astype(np.float16)).to(DEV)
            outs, plans = [], []
            for head in (0, 1):
                gsa.set_config("KS_HEAD", head)
                plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", N, rows, 1).compile().upload("f16", 0)
                assert plan.info()["device_kernel"] == "k_mfma_ks", plan.info()
                outs.append(plan.spmm(B).float().cpu().numpy())
                plans.append(plan)
            gsa.set_config("KS_HEAD", 1)
            np.testing.assert_array_equal(outs[0], outs[1])
            check(outs[1], ofi.spmm_ref(640, N, r, c, v.astype(np.float16).astype(np.float32),
                                        B.cpu().numpy().astype(np.float32), "f64"), "f16")
            plans[1].add_replica()
            Cs = [torch.full((640, N), float("nan"), device=DEV, dtype=torch.float16) for _ in range(3)]
            bat = gsa.Batch([(plans[1], 0, B, Cs[0]), (plans[0], 0, B, Cs[1]), (plans[1], 1, B, Cs[2])], N)
            assert bat.launches() == [3]  # head and record-only entries share the instantiation
            bat.run(torch.cuda.current_stream().cuda_stream)
            for cc in Cs:
                np.testing.assert_array_equal(cc.float().cpu().numpy(), outs[0])
            for p in plans:
                p.device_status()
                p.free()
    finally:
        gsa.set_config("KS_HEAD", 1)
        gsa.set_config("KS_NT", 0)
        gsa.set_config("KS_SPLIT", 0)


@pytest.mark.parametrize("p8", [0, 1])
@pytest.mark.parametrize("rows,split", [(40, 2), (80, 4), (112, 1), (112, 4), (128, 3)])
def test_mfma_ks_four_waves(rows, split, p8, mfma_everywhere):
    """KS_WAVES = 4: 256-thread K-split workgroups with the overlapped LDS layout (two per CU);
    each wave takes every fourth k-step, so the sums differ from the 8-wave kernel's by rounding
    only: oracle parity, a bit-identical relaunch, and one grouped launch of two replicas equal
    to their single launches"""
    need_experiments()
    N = 32
    r, c, v = ds.pruned_weight(640, 2048, 0.7, 12)
    B = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, (2048, N)).astype(np.float16)).to(DEV)
    gsa.set_config("KS_SPLIT", split)
    gsa.set_config("KS_WAVES", 4)
    gsa.set_config("KS_POS8", p8)
    try:
        plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", N, rows, 1).compile().upload("f16", 0)
    finally:
        gsa.set_config("KS_SPLIT", 0)
        gsa.set_config("KS_WAVES", 8)
        gsa.set_config("KS_POS8", 0)
    info = plan.info()
    assert info["device_kernel"] == "k_mfma_ks" and info["lds_waves"] == 4 and info["ksplit"] == split, info
    C = plan.spmm(B).float().cpu().numpy()
    check(C, ofi.spmm_ref(640, N, r, c, v.astype(np.float16).astype(np.float32), B.cpu().numpy().astype(np.float32),
                          "f64"), "f16")
    np.testing.assert_array_equal(plan.spmm(B).float().cpu().numpy(), C)
    plan.add_replica()
    Cs = [torch.full((640, N), float("nan"), device=DEV, dtype=torch.float16) for _ in range(2)]
    bat = gsa.Batch([(plan, 0, B, Cs[0]), (plan, 1, B, Cs[1])], N)
    assert bat.launches() == [2]
    bat.run(torch.cuda.current_stream().cuda_stream)
    for cc in Cs:
        np.testing.assert_array_equal(cc.float().cpu().numpy(), C)
    plan.device_status()
    plan.free()


@pytest.mark.parametrize("split", [2, 4])
def test_mfma_ks_slab_tags_alternate_over_launches(split, mfma_everywhere):
    """The K-split combine's slab tags alternate per launch (epoch in the arrival counter, no
    slab cleared after use): a stale slab from the previous launch must never be taken for a
    fresh one.  Seven launches with a different B each, a replica added after an odd number of
    launches (it copies the slab / counter state), launches alternating between the two, and a
    repeat of the first B at the end: every result equals its first computation bit for bit
    and the oracle within the fp16 tolerance."""
    gsa.set_config("KS_SPLIT", split)
    try:
        r, c, v = ds.pruned_weight(640, 2048, 0.7, 5)
        plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", 32, 80, 1).compile().upload("f16", 0)
        assert plan.info()["device_kernel"] == "k_mfma_ks" and plan.info()["ksplit"] == split
        rng = np.random.default_rng(11)
        Bs = [rng.uniform(-1, 1, (2048, 32)).astype(np.float16) for _ in range(4)]
        vf = v.astype(np.float16).astype(np.float32)
        first = {}
        order = [(0, 0), (1, 0), (2, 0), "add", (3, 1), (0, 0), (1, 1), (2, 0), (3, 0), (0, 1)]
        for step in order:
            if step == "add":
                plan.add_replica()
                continue
            b, rep = step
            C = plan.spmm(torch.from_numpy(Bs[b]).to(DEV), replica=rep).float().cpu().numpy()
            if b in first:
                np.testing.assert_array_equal(C, first[b])
            else:
                check(C, ofi.spmm_ref(640, 32, r, c, vf, Bs[b].astype(np.float32), "f64"), "f16")
                first[b] = C
        plan.free()
    finally:
        gsa.set_config("KS_SPLIT", 0)


def test_mfma_ks_known_answer_and_c2():
    """all-ones known answer bit-exactly, and the C2 shape (80-row blocks, 4 K ranges) against
    a torch fp32 dense product of the same fp16 inputs"""
    M, K, N = 700, 9000, 32
    row, col, _ = ds.random_rows(M, K, 700.0, seed=8, empty_frac=0.1)  # row nnz < 2048: exact in fp16
    plan, C, _ = run(M, K, row, col, np.ones(len(row), np.float32), "block_total", 64, 1, N, "f16",
                     B=np.ones((K, N), np.float16))
    assert plan.info()["device_kernel"] == "k_mfma_ks", plan.info()
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))
    M = K = 5120
    r, c, v = ds.pruned_weight(M, K, 0.7, 13)
    A = torch.zeros((M, K), dtype=torch.float32)
    A[torch.from_numpy(r.astype(np.int64)), torch.from_numpy(c.astype(np.int64))] = torch.from_numpy(v).half().float()
    B = torch.randn((K, N), device=DEV, dtype=torch.float16)
    ref = A.to(DEV) @ B.float()
    plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("block_total", N, 80, 1).compile().upload("f16", 0)
    info = plan.info()
    assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == 4, info
    C = plan.spmm(B).float()
    err = ((C - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
    assert err <= bound("f16", info["device_kernel"]), err
    assert torch.equal(plan.spmm(B * 2).float(), 2 * C)  # linearity, deterministic


def test_c2_driver_plan_block_total_40_against_torch():
    """The plan the driver's C2 line runs: block_total(40,1) on k_mfma_ks with
    two K ranges (128 row blocks of 40 rows = 256 workgroups), at full C2 size against a torch
    fp32 dense product of the same fp16 inputs; a second launch into a NaN-filled C is the
    same bit for bit, linearity is exact, and the device error word stays clear."""
    M = K = 5120
    N = 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 13)
    A = torch.zeros((M, K), dtype=torch.float32)
    A[torch.from_numpy(r.astype(np.int64)), torch.from_numpy(c.astype(np.int64))] = torch.from_numpy(v).half().float()
    B = torch.randn((K, N), device=DEV, dtype=torch.float16)
    ref = A.to(DEV) @ B.float()
    plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("block_total", N, 40, 1).compile().upload("f16", 0)
    info = plan.info()
    assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == 2, info
    C = plan.spmm(B).float()
    err = ((C - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
    assert err <= bound("f16", info["device_kernel"]), err
    C2 = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float16)
    plan.spmm(B, C=C2)
    assert torch.equal(C2.float(), C)
    assert torch.equal(plan.spmm(B * 2).float(), 2 * C)
    plan.device_status()
    plan.free()


def test_ks_combine_timeout_is_reported_at_the_abi(mfma_everywhere):
    """A K-split combine that gives up waiting for a partial slab sets the replica's device
    error word: gs_plan_device_status reports GS_ERR_DEVICE once and clears it (VERDICT r04
    #8).  The timeout path is forced by the experiments build's KS_FORCE_TIMEOUT; the
    default build refuses that switch, and there a clean run reports nothing."""
    r, c, v = ds.pruned_weight(640, 2048, 0.7, 5)
    plan = gsa.Plan.from_coo(640, 2048, r, c, v).run_pipeline("block_total", 32, 80, 1).compile().upload("f16", 0)
    assert plan.info()["device_kernel"] == "k_mfma_ks" and plan.info()["ksplit"] > 1
    B = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, (2048, 32)).astype(np.float16)).to(DEV)
    good = plan.spmm(B)
    plan.device_status()
    from build_flags import EXPERIMENTS
    if not EXPERIMENTS:
        with pytest.raises(gsa.GsError):
            gsa.set_config("KS_FORCE_TIMEOUT", 1)
        plan.free()
        return
    gsa.set_config("KS_FORCE_TIMEOUT", 1)
    try:
        bad = plan.spmm(B)
        with pytest.raises(gsa.GsError) as ei:
            plan.device_status()
        assert ei.value.code == -4 and "timed out" in str(ei.value)
        assert torch.isnan(bad.float()).any()
    finally:
        gsa.set_config("KS_FORCE_TIMEOUT", 0)
    plan.device_status()  # reported once, then clear
    assert torch.equal(plan.spmm(B), good)
    plan.device_status()
    plan.free()


@pytest.mark.parametrize("kernel", ["k_mfma_rows", "k_mfma_ks"])
def test_mfma_unsorted_columns_and_duplicates(kernel, mfma_everywhere):
    """the reference accepts any column order inside a row and its gather kernels
    add repeated coordinates: the matrix-core layouts sort each row and sum
    duplicates"""
    M, K, N = 300, 2100, 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 41)
    rng = np.random.default_rng(3)
    # shuffle the columns inside every row, then repeat 5% of the entries
    order = np.lexsort((rng.random(len(r)), r))
    r, c, v = r[order], c[order], v[order]
    dup = np.sort(rng.choice(len(r), len(r) // 20, replace=False))
    r2 = np.concatenate([r, r[dup]])
    c2 = np.concatenate([c, c[dup]])
    v2 = np.concatenate([v, (0.5 * v[dup]).astype(np.float32)])
    o = np.argsort(r2, kind="stable")
    r2, c2, v2 = r2[o], c2[o], v2[o]
    plan, C, B = run(M, K, r2, c2, v2, "block_total", 20 if kernel == "k_mfma_rows" else 48, 1, N, "f16")
    assert plan.info()["device_kernel"] == kernel
    ref = ofi.spmm_ref(M, N, r2, c2, v2.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    # contract line against the entries as given: a repeated coordinate is rounded to fp16
    # once as its sum (the layout's value), not once per entry, so the tight line does not
    # hold against this reference (~2^-11 of each combined value)
    err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= TOL["f16"], err.max()
    # tight line against the canonical matrix the layout holds: duplicates summed in double,
    # rounded to fp32, then to fp16 (device_layout.cc canonical_rows)
    key = r2.astype(np.int64) * K + c2.astype(np.int64)
    uk, inv = np.unique(key, return_inverse=True)
    vs = np.zeros(len(uk), np.float64)
    np.add.at(vs, inv, v2.astype(np.float64))
    rc, cc = (uk // K).astype(np.uint64), (uk % K).astype(np.uint64)
    vc = vs.astype(np.float32).astype(np.float16).astype(np.float32)
    check(C, ofi.spmm_ref(M, N, rc, cc, vc, B.astype(np.float32), "f64"), "f16", plan)


def test_mfma_non_finite_B_deviation(mfma_everywhere):
    """documented deviation: the matrix-core kernels multiply every
    row block's whole tile, zeros included, so an Inf in B[k, j] makes all of output
    column j non-finite; the reference (and MFMA_TILES=0) only poisons the rows with
    an entry at column k.  The other columns stay finite either way."""
    M, K, N = 200, 640, 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 43)
    B = np.random.default_rng(5).uniform(-1, 1, (K, N)).astype(np.float16)
    k = 77
    B[k, 3] = np.inf
    plan, C, _ = run(M, K, r, c, v, "block_total", 20, 1, N, "f16", B=B)
    assert plan.info()["device_kernel"] == "k_mfma_rows"
    has_k = np.zeros(M, bool)
    has_k[r[c == k].astype(np.int64)] = True
    assert not np.isfinite(C[:, 3]).any()               # the whole column (reference: rows has_k only)
    assert np.isfinite(np.delete(C, 3, axis=1)).all()   # other columns untouched
    try:
        gsa.set_config("MFMA_TILES", 0)
        plan0, C0, _ = run(M, K, r, c, v, "block_total", 20, 1, N, "f16", B=B)
        assert not plan0.info()["device_kernel"].startswith("k_mfma")
        np.testing.assert_array_equal(np.isfinite(C0[:, 3]), ~has_k)  # reference semantics
    finally:
        gsa.set_config("MFMA_TILES", 1)


def test_mfma_rows_known_answer_and_fallback(mfma_everywhere):
    M, K, N = 700, 9000, 32
    row, col, _ = ds.random_rows(M, K, 60.0, seed=8, empty_frac=0.1)
    plan, C, _ = run(M, K, row, col, np.ones(len(row), np.float32), "block_total", 20, 1, N, "f16",
                     B=np.ones((K, N), np.float16))
    assert plan.info()["lds_stage"] == 2
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))
    # another dense width than the plan's runs the gather kernel
    B2 = np.random.default_rng(2).uniform(-1, 1, (K, 24)).astype(np.float16)
    C2 = plan.spmm(torch.from_numpy(B2).to(DEV)).float().cpu().numpy()
    ref2 = ofi.spmm_ref(M, 24, row, col, np.ones(len(row), np.float32), B2.astype(np.float32), "f64")
    check(C2, ref2, "f16")


def test_mfma_rows_selection():
    M, K, N = 400, 2000, 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 5)
    plan, _, _ = run(M, K, r, c, v, "block_total", 20, 1, N, "f16")
    assert plan.info()["lds_stage"] == 2          # 30% dense: matrix cores
    plan, _, _ = run(M, K, r, c, v, "block_total", 20, 1, N, "f32")
    assert plan.info()["lds_stage"] == 0          # fp32: CUDA-core kernels
    rr, cc, vv = ds.random_rows(M, K, 10.0, seed=6)
    plan, _, _ = run(M, K, rr, cc, vv, "block_total", 20, 1, N, "f16")
    assert plan.info()["lds_stage"] == 0          # 0.5% dense: too sparse for tiles
    try:
        gsa.set_config("MFMA_TILES", 0)
        plan, _, _ = run(M, K, r, c, v, "tblock_warp_total", 20, 2, N, "f16")
        assert plan.info()["lds_stage"] == 1
    finally:
        gsa.set_config("MFMA_TILES", 1)


@pytest.mark.parametrize("ks", [1, 2, 3])
def test_mfma_rows_ksplit_combine(ks, mfma_everywhere):
    """K ranges per row block combined through fp32 slabs by the last arriving
    workgroup: same result (within fp16 output rounding) for every split, exact
    known answer, and the arrival counters reset for the next launch"""
    M, K, N = 400, 6000, 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 31)
    try:
        gsa.set_config("MFMA_KS", 0)  # the k_mfma_rows split (k_mfma_ks: test_mfma_ks_*)
        gsa.set_config("MFMA_KSPLIT", ks)
        plan, C, B = run(M, K, r, c, v, "block_total", 40, 1, N, "f16")
        info = plan.info()
        assert info["lds_stage"] == 2 and info["ksplit"] == ks, info
        ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
        check(C, ref, "f16")
        Bt = torch.from_numpy(B).to(DEV)
        again = [plan.spmm(Bt).float().cpu().numpy() for _ in range(3)]
        for a in again:
            np.testing.assert_array_equal(a, C)   # deterministic, counters reset
        plan.add_replica()
        np.testing.assert_array_equal(plan.spmm(Bt, replica=1).float().cpu().numpy(), C)
        _, ones, _ = run(M, K, r, c, np.ones(len(r), np.float32), "block_total", 40, 1, N, "f16",
                         B=np.ones((K, N), np.float16))
        nnz_row = np.bincount(r.astype(np.int64), minlength=M).astype(np.float32)
        np.testing.assert_array_equal(ones, np.repeat(nnz_row[:, None], N, axis=1))
    finally:
        gsa.set_config("MFMA_KSPLIT", 0)


# merge-path plans (A11, C4): rows crossing waves, waves closing rows exactly at their
# end, long runs of empty rows (leading, inner, trailing), one-nnz rows
def merge_cases():
    rng = np.random.default_rng(21)
    M, K = 5000, 700
    lens = rng.integers(0, 4, M)
    lens[:37] = 0                      # leading empty rows
    lens[-101:] = 0                    # trailing empty rows
    lens[1000:1400] = 0                # inner run of empty rows
    lens[2000] = 9000                  # a row crossing many waves
    lens[2001] = 513
    rows = np.repeat(np.arange(M, dtype=np.uint64), lens)
    cols = (rng.integers(0, K, len(rows))).astype(np.uint64)
    yield "mixed", M, K, rows, cols, rng.uniform(-1, 1, len(rows)).astype(np.float32)
    r, c, v = ds.rmat(4096, 60000, seed=3)
    yield "rmat", 4096, 4096, r, c, v
    rows = np.arange(2048, dtype=np.uint64)  # one nnz per row
    yield "diag", 2048, 2048, rows, rows.copy(), np.linspace(-1, 1, 2048).astype(np.float32)


@pytest.fixture(params=[0, 1], ids=["k_merge_path", "k_merge_rows"])
def merge_walk(request):
    """both merge-path walks (MP_ROWS fixes the kernel at upload; k_merge_rows is an
    experiments-build kernel)"""
    need_experiments(request.param == 1)
    gsa.set_config("MP_ROWS", request.param)
    yield "k_merge_rows" if request.param else "k_merge_path"
    gsa.set_config("MP_ROWS", 0)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 3, 64])
@pytest.mark.parametrize("ws,level", [(1024, 1), (37, 1), (1, 3), (512, 2), (100000, 1)])
def test_merge_path_matches_oracle(ws, level, N, dtype, merge_walk):
    for case, M, K, row, col, val in merge_cases():
        plan, C, B = run(M, K, row, col, val, "merge_path", ws, level, N, dtype)
        assert plan.info()["kernel_name"].startswith("k_merge_path"), plan.info()["kernel_name"]
        assert plan.info()["device_kernel"] == merge_walk
        v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        check(C, ref, dtype, plan)


@pytest.mark.parametrize("parts,hub", [(2, 0), (4, 0), (8, 0), (2, 300)])
@pytest.mark.parametrize("N", [8, 3, 32])
@pytest.mark.parametrize("ws", [512, 37])
def test_merge_path_column_partitions(parts, hub, N, ws):
    """MP_COL_PARTS (fp32 merge-path plans with MP_COL_PERM): the degree-ranked columns dealt
    over P partitions, one k_merge_path pass per partition over its own CSR and wave ranges,
    the partitions' fp32 outputs added to C in partition order: against the oracle, relaunches
    into NaN-filled C bit for bit (the chains' counters re-arm), a replica the same bits"""
    M = 3000
    row, col, val = ds.rmat(M, 60000, seed=9)
    # a few rows over many waves and empty rows: chains inside a partition
    row = np.concatenate([row, np.full(4000, 1500, np.uint64)])
    col = np.concatenate([col, np.arange(4000, dtype=np.uint64) % M])
    val = np.concatenate([val, np.linspace(-1, 1, 4000).astype(np.float32)])
    key = np.unique(row.astype(np.int64) * M + col.astype(np.int64), return_index=True)[1]
    row, col, val = row[key], col[key], val[key]
    B = np.random.default_rng(4).uniform(-1, 1, (M, N)).astype(np.float32)
    gsa.set_config("MP_COL_PERM", 1)
    gsa.set_config("MP_COL_PARTS", parts)
    gsa.set_config("MP_HUB_COLS", hub)  # (2, 300): the 300 densest columns, then the rest
    try:
        plan = gsa.Plan.from_coo(M, M, row, col, val).run_pipeline("merge_path", N, ws, 1).compile().upload("f32", 0)
    finally:
        gsa.set_config("MP_COL_PARTS", 0)
        gsa.set_config("MP_HUB_COLS", 0)
        gsa.set_config("MP_COL_PERM", -1)
    assert plan.info()["device_kernel"] == "k_merge_path"
    Bt = torch.from_numpy(B).to(DEV)
    C = plan.spmm(Bt)
    torch.cuda.synchronize()
    check(C.cpu().numpy(), ofi.spmm_ref(M, N, row, col, val, B, "f64"), "f32", plan)
    plan.add_replica()
    for rep in (0, 1, 0):
        C2 = torch.full((M, N), float("nan"), device=DEV)
        plan.spmm(Bt, C=C2, replica=rep)
        torch.cuda.synchronize()
        assert torch.equal(C2, C)
    plan.free()


@pytest.mark.parametrize("variant", [{}, {"MP_PERM_SCATTER": 1}, {"MP_PERM_HOT": 300}])
@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 3])
def test_merge_path_column_permutation_is_exact(N, dtype, variant):
    """MP_COL_PERM renumbers a merge-path plan's columns by degree on the device and gathers B
    into that order per launch (k_permute_rows): only where B rows sit in memory changes, the
    order of every row's entries does not, so C is bit-identical to the unpermuted plan's (and
    matches the oracle); replicas carry their own permuted B"""
    M = 3000
    row, col, val = ds.rmat(M, 60000, seed=9)
    npdt = np.float16 if dtype == "f16" else np.float32
    B = np.random.default_rng(4).uniform(-1, 1, (M, N)).astype(npdt)
    outs = []
    for perm in (0, 1):
        gsa.set_config("MP_COL_PERM", perm)
        for k, v in variant.items():
            gsa.set_config(k, v)
        try:
            plan = gsa.Plan.from_coo(M, M, row, col, val).run_pipeline("merge_path", N, 512, 1).compile().upload(dtype, 0)
        finally:
            gsa.set_config("MP_COL_PERM", -1)
            for k in variant:
                gsa.set_config(k, 0)
        plan.add_replica()
        Bt = torch.from_numpy(B).to(DEV)
        C0 = plan.spmm(Bt).float().cpu().numpy()
        C1 = plan.spmm(Bt, replica=1).float().cpu().numpy()
        np.testing.assert_array_equal(C0, C1)
        outs.append(C0)
        plan.free()
    np.testing.assert_array_equal(outs[0], outs[1])
    vv = val.astype(npdt).astype(np.float32)
    check(outs[1], ofi.spmm_ref(M, N, row, col, vv, B.astype(np.float32), "f64"), dtype)


def test_merge_path_deterministic_and_no_stale_state(merge_walk):
    """two launches give bit-identical C (no floating-point atomics: a split row's partials
    are combined in wave order by the last arriver on an integer arrival counter, and the
    carries are re-written every launch), and C's prior content (NaN) is fully overwritten,
    empty rows included"""
    _, M, K, row, col, val = next(merge_cases())
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("merge_path", 8, 64, 1).compile().upload("f32", 0)
    B = torch.from_numpy(np.random.default_rng(4).uniform(-1, 1, (K, 8)).astype(np.float32)).to(DEV)
    C1 = torch.full((M, 8), float("nan"), device=DEV)
    plan.spmm(B, C=C1)
    C2 = plan.spmm(B)
    torch.cuda.synchronize()
    assert not torch.isnan(C1).any()
    assert torch.equal(C1, C2)


def test_loaded_plan_file_computes_the_same(tmp_path):
    """§8f rank 4: a plan loaded from its binary file gives bit-identical C (merge path,
    matrix-core row blocks)"""
    for name, p0, p1, dtype, N in [("merge_path", 256, 1, "f32", 8), ("tblock_warp_total", 20, 2, "f16", 32)]:
        M, K = 640, 700
        r, c, v = ds.random_rows(M, K, 40.0, seed=3, empty_frac=0.1)
        plan, C, B = run(M, K, r, c, v, name, p0, p1, N, dtype)
        f = tmp_path / f"{name}.gsplan"
        plan.save(f)
        q = gsa.Plan.load(f).upload(dtype, 0)
        C2 = q.spmm(torch.from_numpy(B).to(DEV))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C, C2.float().cpu().numpy())


def test_autotune_picks_a_timed_variant(tmp_path):
    from generalsparse_amd.autotune import autotune
    M, K = 1024, 1024
    r, c, v = ds.rmat(1024, 20000, seed=5)
    f = tmp_path / "best.gsplan"
    plan, res = autotune(M, K, r, c, v, 8, "f32", reps=5, rotation_mb=16, save_path=f)
    timed = {k: t for k, t in res.items() if isinstance(t, float)}
    assert timed and f.exists()
    B = np.random.default_rng(0).uniform(-1, 1, (K, 8)).astype(np.float32)
    C = plan.spmm(torch.from_numpy(B).to(DEV))
    torch.cuda.synchronize()
    check(C.float().cpu().numpy(), ofi.spmm_ref(M, 8, r, c, v, B, "f64"), "f32")


def test_autotune_on_c2_finds_the_measured_plan():
    """the product's search (autotune's default candidates, the same table
    bench.py searches) on C2 returns the plan the C2 line measures: k_mfma_ks with 2 K ranges
    (block_total(40,1), with or without KS_NT), and that plan is parity-green"""
    from generalsparse_amd.autotune import autotune
    M = K = 5120
    N = 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 13)
    plan, res = autotune(M, K, r, c, v, N, "f16", reps=50, rotation_mb=640)
    info = plan.info()
    best = min((t, k) for k, t in res.items() if isinstance(t, float))
    assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == 2, (info, res)
    assert best[1].startswith("block_total(40,1)"), res
    B = torch.randn((K, N), device=DEV, dtype=torch.float16)
    A = torch.zeros((M, K), dtype=torch.float32)
    A[torch.from_numpy(r.astype(np.int64)), torch.from_numpy(c.astype(np.int64))] = torch.from_numpy(v).half().float()
    ref = A.to(DEV) @ B.float()
    C = plan.spmm(B).float()
    err = ((C - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
    assert err <= bound("f16", info["device_kernel"]), err
    plan.free()


# §8f rank 3: one kernel per sub-matrix of a row division, run in sequence by gs_spmm
SUB_MIXES = [
    ("merge_path", 64, 1, "thread_total", 4, 1),
    ("tblock_warp_total", 16, 2, "warp_total", 0, 1),
    ("balanced_warp_total", 256, 1, "block_total", 0, 1),
    ("thread_bit_map", 4, 1, "warp_segment", 4, 1),
]


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 32])
@pytest.mark.parametrize("mix", SUB_MIXES, ids=lambda m: f"{m[0]}+{m[3]}")
def test_sub_matrix_kernels_match_oracle(mix, N, dtype):
    M, K = 900, 400
    r, c, v = ds.random_rows(M, K, 14.0, seed=7, empty_frac=0.1)
    keep = (r < 300) | (r >= 450)  # interval [300, 450) without nonzeros: zeroed by the executor
    r, c, v = r[keep], c[keep], v[keep]
    plan = gsa.Plan.from_coo(M, K, r, c, v)
    subs = plan.divide_rows(150)
    assert len(subs) == 5
    for i, s in enumerate(subs):
        name, p0, p1 = mix[0:3] if i % 2 == 0 else mix[3:6]
        plan.run_pipeline(name, N, p0, p1, sub=s)
    plan.compile().upload(dtype, 0)
    assert plan.info()["n_kernels"] == 5
    npdt = np.float16 if dtype == "f16" else np.float32
    B = np.random.default_rng(8).uniform(-1, 1, (K, N)).astype(npdt)
    C = torch.full((M, N), float("nan"), dtype=torch.float16 if dtype == "f16" else torch.float32, device=DEV)
    plan.spmm(torch.from_numpy(B).to(DEV), C=C)
    torch.cuda.synchronize()
    Cn = C.float().cpu().numpy()
    assert not np.isnan(Cn).any()
    check(Cn, ofi.spmm_ref(M, N, r, c, v, B, "f64"), dtype)


def test_divided_plan_file_computes_the_same(tmp_path):
    """a divided plan loaded from its binary file (every sub-matrix's kernel) gives
    bit-identical C"""
    M, K, N = 900, 400, 32
    r, c, v = ds.random_rows(M, K, 14.0, seed=9, empty_frac=0.1)
    keep = (r < 300) | (r >= 450)
    r, c, v = r[keep], c[keep], v[keep]
    plan = gsa.Plan.from_coo(M, K, r, c, v)
    for i, s in enumerate(plan.divide_rows(150)):
        plan.run_pipeline("merge_path" if i % 2 else "tblock_warp_total", N, 64 if i % 2 else 16, 1 if i % 2 else 2, sub=s)
    plan.compile().upload("f16", 0)
    f = tmp_path / "divided.gsplan"
    plan.save(f)
    q = gsa.Plan.load(f).upload("f16", 0)
    B = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, (K, N)).astype(np.float16)).to(DEV)
    C1 = torch.full((M, N), float("nan"), dtype=torch.float16, device=DEV)
    C2 = torch.full((M, N), float("nan"), dtype=torch.float16, device=DEV)
    plan.spmm(B, C=C1)
    q.spmm(B, C=C2)
    torch.cuda.synchronize()
    assert not torch.isnan(C2).any()
    assert torch.equal(C1, C2)


@pytest.mark.parametrize("groups", [1, 0])
@pytest.mark.parametrize("N", [8, 32])
def test_warp_rows_grouped_passes(groups, N):
    """k_warp_rows with several short rows of a BMW per wave pass (WARP_ROWS_GROUPS, the
    software-pipelined path; C1-like rows of ~37 nonzeros in BMWs of 8 rows) and without:
    both match the oracle (LDS staging off: at fp32 N = 32 these BMWs of 8 rows would run
    k_lds_rows_rs)"""
    M, K = 3000, 2000
    row, col, val = ds.random_rows(M, K, 37.0, seed=6, empty_frac=0.05)
    gsa.set_config("WARP_ROWS_GROUPS", groups)
    gsa.set_config("LDS_STAGE_B", 0)
    try:
        plan, C, B = run(M, K, row, col, val, "tblock_warp_total", 32, 8, N, "f32")
    finally:
        gsa.set_config("WARP_ROWS_GROUPS", 1)
        gsa.set_config("LDS_STAGE_B", 1)
    assert plan.info()["device_kernel"].startswith("k_warp_rows"), plan.info()["device_kernel"]
    check(C, ofi.spmm_ref(M, N, row, col, val, B, "f64"), "f32")
    plan.free()


@pytest.mark.parametrize("N", [16, 32, 64])
@pytest.mark.parametrize("pipe", MFMA_PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_mfma_rows_counter_handoffs(pipe, N, mfma_everywhere):
    """k_mfma_rows with MFMA_FLAGS (the roles hand buffers over through LDS counters, no
    per-chunk barrier): oracle parity, determinism, and the C2 shape against torch"""
    need_experiments()
    name, p0, p1 = pipe
    gsa.set_config("MFMA_GLDS", 1)
    gsa.set_config("MFMA_FLAGS", 1)
    try:
        used = []
        for case, M, K, row, col, val in mfma_cases():
            plan, C, B = run(M, K, row, col, val, name, p0, p1, N, "f16")
            used.append(plan.info()["device_kernel"])
            ref = ofi.spmm_ref(M, N, row, col, val.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
            check(C, ref, "f16")
            np.testing.assert_array_equal(plan.spmm(torch.from_numpy(B).to(DEV)).float().cpu().numpy(), C)
            plan.free()
        if N == 32 and p0 <= 32:
            assert "k_mfma_rows" in used, used
    finally:
        gsa.set_config("MFMA_FLAGS", 0)


@pytest.mark.parametrize("N", [8, 32, 128])
@pytest.mark.parametrize("pipe", KS_PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_mfma_ks_16_waves(pipe, N, mfma_everywhere):
    """k_mfma_ks with KS_WAVES=16 (twice the waves per workgroup where their stages fit LDS):
    oracle parity, determinism of the K-range combine"""
    need_experiments()
    name, p0, p1 = pipe
    gsa.set_config("KS_WAVES", 16)
    try:
        waves = []
        for case, M, K, row, col, val in mfma_cases():
            plan, C, B = run(M, K, row, col, val, name, p0, p1, N, "f16")
            info = plan.info()
            if info["device_kernel"] == "k_mfma_ks":
                waves.append(info["lds_waves"])
            ref = ofi.spmm_ref(M, N, row, col, val.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
            check(C, ref, "f16")
            np.testing.assert_array_equal(plan.spmm(torch.from_numpy(B).to(DEV)).float().cpu().numpy(), C)
            plan.free()
        if N <= 32:  # (at N = 128 a 64-row block's 16 wave stages exceed LDS: 8 waves)
            assert 16 in waves, waves
    finally:
        gsa.set_config("KS_WAVES", 8)


def test_batch_grouped_launch_matches_single_launches():
    """gs_spmm_batch: consecutive K-split entries of one instantiation run as one grouped
    launch (k_mfma_ks_group); every C equals its single launch bit for bit, across group
    boundaries (another kernel family in between, a (plan, replica) repeated, more than 32
    entries)"""
    N = 32
    mats = [ds.pruned_weight(700, 3000, 0.7, 41), ds.pruned_weight(700, 3000, 0.7, 42)]
    plans = []
    for r, c, v in mats:
        p = gsa.Plan.from_coo(700, 3000, r, c, v).run_pipeline("block_total", N, 80, 1).compile().upload("f16", 0)
        assert p.info()["device_kernel"] == "k_mfma_ks", p.info()
        for _ in range(35):
            p.add_replica()
        plans.append(p)
    r, c, v = ds.random_rows(500, 3000, 20.0, seed=43)
    pg = gsa.Plan.from_coo(500, 3000, r, c, v).run_pipeline("warp_segment", N, 4, 1).compile().upload("f16", 0)
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    Bs = [(torch.rand((3000, N), device=DEV, generator=g) * 2 - 1).half() for _ in range(3)]
    entries = [(plans[0], 0, Bs[0]), (plans[0], 1, Bs[1]), (plans[1], 0, Bs[2]), (pg, 0, Bs[0]), (plans[1], 1, Bs[0]),
               (plans[0], 1, Bs[2]), (plans[1], 2, Bs[1])]
    entries += [(plans[k % 2], 3 + k // 2, Bs[k % 3]) for k in range(40)]
    Cs = [torch.full((p.info()["rows"], N), float("nan"), device=DEV, dtype=torch.float16) for (p, _, _) in entries]
    gsa.Batch([(p, rep, b, cc) for (p, rep, b), cc in zip(entries, Cs)], N).run(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for (p, rep, b), cc in zip(entries, Cs):
        ref = p.spmm(b, replica=rep)
        torch.cuda.synchronize()
        assert torch.equal(cc, ref), (rep,)
    for p in plans + [pg]:
        p.free()


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("chunks", [1, 2, 3])
@pytest.mark.parametrize("p0,p1", [(32, 8), (8, 8), (16, 4)])
def test_warp_rows_chunks_per_pass(p0, p1, chunks, dtype):
    """k_warp_rows grouped passes with WARP_ROWS_CHUNKS SCF-chunks per slot (all A loads, then all
    gathers of a pass in flight): every case of coo_cases plus a C1-like matrix (Poisson rows of
    ~37 nonzeros, some past the pass capacity) against the oracle"""
    old = gsa.get_config("WARP_ROWS_CHUNKS")
    gsa.set_config("WARP_ROWS_CHUNKS", chunks)
    try:
        cases = list(coo_cases())
        cases.append(("c1_like", 4000, 3000, *ds.random_rows(4000, 3000, 37.4, seed=18)))
        r, c, v = ds.random_rows(800, 3000, 37.4, seed=19)
        keep = ((r % 97) != 5) & (r != 7)  # some empty rows; row 7 rebuilt as a 300-nonzero row
        r2 = np.concatenate([r[keep], np.full(300, 7, r.dtype)])
        c2 = np.concatenate([c[keep], np.arange(300, dtype=c.dtype) * 9])
        v2 = np.concatenate([v[keep], np.ones(300, v.dtype)])
        o = np.lexsort((c2, r2))
        cases.append(("c1_long_rows", 800, 3000, r2[o], c2[o], v2[o]))
        for case, M, K, row, col, val in cases:
            plan, C, B = run(M, K, row, col, val, "tblock_warp_total", p0, p1, 8, dtype)
            v32 = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val.astype(np.float32)
            ref = ofi.spmm_ref(M, 8, row, col, v32, B.astype(np.float32), "f64")
            check(C, ref, dtype, plan)
            plan.free()
    finally:
        gsa.set_config("WARP_ROWS_CHUNKS", old)


@pytest.mark.parametrize("rows,split,grid", [(40, 2, 256), (40, 4, 256), (80, 4, 256), (40, 4, 64), (48, 3, 7)])
def test_mfma_ks_persistent_grid_is_exact(rows, split, grid):
    """KS_PERSIST (experiments build): a persistent grid pulling (row block,
    K range) units from per-XCD heads computes the same bits as the static k_mfma_ks launch
    (the K-range combine is the same tickets + tagged slabs in q order), relaunch after
    relaunch (the heads re-arm), also with fewer workgroups than XCD heads (stealing)"""
    need_experiments()
    M = K = 5120 if grid >= 64 else 1536
    N = 32
    r, c, v = ds.pruned_weight(M, K, 0.7, 13)
    B = torch.randn((K, N), device=DEV, dtype=torch.float16)
    outs = []
    for persist in (0, grid):
        gsa.set_config("KS_SPLIT", split)
        gsa.set_config("KS_PERSIST", persist)
        gsa.set_config("KS_NT", 1)
        try:
            plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("block_total", N, rows, 1).compile().upload("f16", 0)
        finally:
            gsa.set_config("KS_SPLIT", 0)
            gsa.set_config("KS_PERSIST", 0)
            gsa.set_config("KS_NT", 0)
        info = plan.info()
        assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == split, info
        for _ in range(3):
            C = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float16)
            plan.spmm(B, C=C)
            torch.cuda.synchronize()
            outs.append(C.clone())
        plan.device_status()
        plan.free()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    vf = v.astype(np.float16).astype(np.float32)
    check(outs[0].float().cpu().numpy(), ofi.spmm_ref(M, N, r, c, vf, B.float().cpu().numpy(), "f64"), "f16")
