"""GPU parity of the 2:4 sparse-matrix-core path (k_nm_mfma, SURVEY.md §8a A10,
BASELINE.json configs[2]): col-direction plans whose rows are 2:4 panels.

Checked against the oracle's fp64 SpMM of the same fp16 inputs (tolerance 1e-1
relative to max(1, |ref|), north_star), the reference's all-ones known answer
bit-exactly, linearity exactly, the row-chunk kernel of the same plan, and at
C3 scale against a torch fp32 dense matmul."""
import numpy as np
import pytest

import oracle_ffi as ofi

torch = pytest.importorskip("torch")
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402
from build_flags import need_experiments  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def plan_for(M, K, row, col, val, N, p0=32):
    return gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("col_direction_nm", N, p0, 1).compile().upload("f16", 0)


def spmm(plan, B):
    C = plan.spmm(torch.from_numpy(B).to(DEV))
    torch.cuda.synchronize()
    return C.float().cpu().numpy()


def check(C, ref, tol=2.0 ** -9):
    """k_nm_mfma / k_row_chunks accumulate in fp32 and round to fp16 once: the tight fp16 line
    (tests/tolerance.py) inside the contract's 1e-1"""
    err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= tol, f"max rel err {err.max()} > {tol}"


def thinned(M, K, seed, keep=0.6, empty_rows=()):
    """2:4 rows with a random share of the entries dropped (groups of 0/1 entries)
    and some rows emptied."""
    r, c, v = ds.two_four(M, K, seed)
    rng = np.random.default_rng(seed + 1)
    m = rng.random(len(r)) < keep
    for e in empty_rows:
        m &= r != e
    return r[m], c[m], v[m]


SHAPES = [(128, 256), (96, 512), (200, 1000), (333, 772), (64, 64), (1, 4096), (1792, 768)]


@pytest.mark.parametrize("N", [8, 16, 32, 64, 128])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: f"{s[0]}x{s[1]}")
def test_nm_matches_oracle(shape, N):
    """N = 8 runs one half-used 16-column tile (k_nm_mfma's NG = 8)"""
    M, K = shape
    r, c, v = ds.two_four(M, K, 30 + M)
    plan = plan_for(M, K, r, c, v, N)
    assert plan.info()["lds_stage"] == 3, plan.info()
    B = np.random.default_rng(M + K).uniform(-1, 1, (K, N)).astype(np.float16)
    ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    check(spmm(plan, B), ref)


@pytest.mark.parametrize("N", [8, 32, 128])
def test_nm_thinned_and_empty_rows(N):
    M, K = 300, 1536
    r, c, v = thinned(M, K, 5, empty_rows=(0, 7, 299, 150))
    plan = plan_for(M, K, r, c, v, N)
    assert plan.info()["lds_stage"] == 3
    B = np.random.default_rng(1).uniform(-1, 1, (K, N)).astype(np.float16)
    ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    C = spmm(plan, B)
    check(C, ref)
    assert np.all(C[[0, 7, 150, 299]] == 0)


@pytest.mark.parametrize("N", [8, 128])
def test_nm_known_answer(N):
    # reference known answer (code_generator.cc:633-637): all-ones A and B => C[i][j] = nnz(row i)
    M, K = 257, 2048
    r, c, _ = thinned(M, K, 9, keep=0.8)
    plan = plan_for(M, K, r, c, np.ones(len(r), np.float32), N)
    C = spmm(plan, np.ones((K, N), np.float16))
    nnz_row = np.bincount(r.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))


def test_nm_linearity_and_determinism():
    M, K, N = 384, 2048, 64
    r, c, v = ds.two_four(M, K, 3)
    plan = plan_for(M, K, r, c, v, N)
    B = np.random.default_rng(2).uniform(-1, 1, (K, N)).astype(np.float16)
    C1 = spmm(plan, B)
    C2 = spmm(plan, (B.astype(np.float32) * 2).astype(np.float16))
    np.testing.assert_array_equal(C2, 2 * C1)
    np.testing.assert_array_equal(spmm(plan, B), C1)


def test_nm_agrees_with_row_chunk_kernel():
    M, K, N = 256, 1024, 32
    r, c, v = ds.two_four(M, K, 12)
    B = np.random.default_rng(4).uniform(-1, 1, (K, N)).astype(np.float16)
    C_nm = spmm(plan_for(M, K, r, c, v, N), B)
    gsa.set_config("NM_MFMA", 0)
    try:
        p = plan_for(M, K, r, c, v, N)
        assert p.info()["lds_stage"] == 0 and p.info()["kernel_name"].startswith("k_row_chunks")
        C_rc = spmm(p, B)
    finally:
        gsa.set_config("NM_MFMA", 1)
    check(C_nm, C_rc, 2e-2)


def test_not_two_four_falls_back():
    M, K, N = 64, 512, 32
    r, c, v = ds.two_four(M, K, 1)
    # a third entry in the first group of row 5
    taken = set(c[r == 5][:2].tolist())
    extra = next(x for x in range(4) if x not in taken)
    r = np.concatenate([r, np.array([5], np.uint64)])
    c = np.concatenate([c, np.array([extra], np.uint64)])
    v = np.concatenate([v, np.array([0.5], np.float32)])
    o = np.lexsort((c, r))
    r, c, v = r[o], c[o], v[o]
    plan = plan_for(M, K, r, c, v, N)
    assert plan.info()["lds_stage"] == 0
    B = np.random.default_rng(0).uniform(-1, 1, (K, N)).astype(np.float16)
    ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    check(spmm(plan, B), ref)


def test_nm_other_widths_refused():
    M, K = 64, 256
    r, c, v = ds.two_four(M, K, 2)
    plan = plan_for(M, K, r, c, v, 32)
    with pytest.raises(gsa.GsError):
        plan.spmm(torch.zeros((K, 48), device=DEV, dtype=torch.float16))


def test_nm_c3_scale_against_dense():
    # BASELINE.json configs[2] shape at half height (14336 x 7168, N = 128) vs torch fp32
    M, K, N = 14336, 7168, 128
    r, c, v = ds.two_four(M, K, 30)
    plan = plan_for(M, K, r, c, v, N)
    assert plan.info()["lds_stage"] == 3
    v16 = torch.from_numpy(v.astype(np.float16).astype(np.float32))
    A = torch.zeros((M, K), dtype=torch.float32)
    A[torch.from_numpy(r.astype(np.int64)), torch.from_numpy(c.astype(np.int64))] = v16
    B = torch.rand((K, N), dtype=torch.float32).mul_(2).sub_(1).half()
    ref = (A.to(DEV) @ B.float().to(DEV)).cpu().numpy()
    C = plan.spmm(B.to(DEV))
    torch.cuda.synchronize()
    check(C.float().cpu().numpy(), ref)


@pytest.mark.parametrize("ks,split", [(0, 0), (1, 1), (1, 3), (1, 0)])
@pytest.mark.parametrize("N", [32, 128])
@pytest.mark.parametrize("shape", [(333, 772), (520, 3000), (1, 4096)], ids=lambda s: f"{s[0]}x{s[1]}")
def test_nm_ks_and_classic_kernels(shape, N, ks, split):
    """k_nm_mfma_ks (256-row workgroups, K split over NM_SPLIT ranges, slab combine by the
    last arriver) and the classic k_nm_mfma: oracle parity, determinism, replicas"""
    need_experiments(ks == 1)
    old = {k: gsa.get_config(k) for k in ("NM_KS", "NM_SPLIT")}
    try:
        gsa.set_config("NM_KS", ks)
        gsa.set_config("NM_SPLIT", split)
        M, K = shape
        r, c, v = thinned(M, K, 70 + M, keep=0.8, empty_rows=(0, M // 2) if M > 2 else ())
        plan = plan_for(M, K, r, c, v, N)
        v4 = gsa.get_config("NM_V4")
        classic = "k_nm_mfma4" if K % 256 == 0 and ((v4 < 0 and N == 128) or (v4 > 0 and N in (64, 128))) else "k_nm_mfma"
        assert plan.info()["device_kernel"] == ("k_nm_mfma_ks" if ks else classic), plan.info()
        B = np.random.default_rng(M + N).uniform(-1, 1, (K, N)).astype(np.float16)
        ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
        C = spmm(plan, B)
        check(C, ref)
        np.testing.assert_array_equal(spmm(plan, B), C)  # counters re-armed, same order
        plan.add_replica()
        C1 = plan.spmm(torch.from_numpy(B).to(DEV), replica=1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C1.float().cpu().numpy(), C)
        plan.free()
    finally:
        for k, val in old.items():
            gsa.set_config(k, val)


@pytest.mark.parametrize("split", [0, 1, 2, 3])
@pytest.mark.parametrize("N", [64, 128])
@pytest.mark.parametrize("shape", [(512, 1024), (333, 2048), (1, 4096), (1000, 768), (256, 512)],
                         ids=lambda s: f"{s[0]}x{s[1]}")
def test_nm4_matches_oracle(shape, N, split):
    """k_nm_mfma4 (256-row workgroups of four row groups x two k-phases, K split over NM_SPLIT
    ranges, B by LDS-DMA, tagged-slab combine): oracle parity (rows not a multiple of 256, empty
    rows, one-chunk ranges), bit-identical relaunch and replica, and agreement with k_nm_mfma
    within the fp16 rounding of the final store"""
    need_experiments()
    M, K = shape
    old = {k: gsa.get_config(k) for k in ("NM_V4", "NM_SPLIT")}
    try:
        gsa.set_config("NM_SPLIT", split)
        r, c, v = thinned(M, K, 90 + M, keep=0.85, empty_rows=(0, M // 2) if M > 2 else ())
        gsa.set_config("NM_V4", 1)
        plan = plan_for(M, K, r, c, v, N)
        info = plan.info()
        assert info["device_kernel"] == "k_nm_mfma4", info
        B = np.random.default_rng(M + N + split).uniform(-1, 1, (K, N)).astype(np.float16)
        ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
        C = spmm(plan, B)
        check(C, ref)
        np.testing.assert_array_equal(spmm(plan, B), C)  # counters re-armed, slab tags alternate
        plan.add_replica()
        C1 = plan.spmm(torch.from_numpy(B).to(DEV), replica=1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(C1.float().cpu().numpy(), C)
        plan.device_status()
        plan.free()
        gsa.set_config("NM_V4", 0)
        p2 = plan_for(M, K, r, c, v, N)
        assert p2.info()["device_kernel"] == "k_nm_mfma"
        C2 = spmm(p2, B)
        p2.free()
        np.testing.assert_allclose(C, C2, rtol=2e-3, atol=2e-3)
    finally:
        for k, val in old.items():
            gsa.set_config(k, val)


@pytest.mark.parametrize("N", [8, 32, 128])
@pytest.mark.parametrize("shape", [(333, 772), (1792, 768), (1, 4096)], ids=lambda s: f"{s[0]}x{s[1]}")
def test_nm_nontemporal_loads_bit_identical(shape, N):
    """NM_NT (default 1: A's panel blocks by non-temporal loads) changes the cache policy of
    the loads only: the result equals the NM_NT=0 kernel's bit for bit, and the oracle's"""
    M, K = shape
    r, c, v = ds.two_four(M, K, 70 + M)
    B = np.random.default_rng(M * N).uniform(-1, 1, (K, N)).astype(np.float16)
    out = {}
    old = gsa.get_config("NM_NT")
    try:
        for nt in (0, 1):
            gsa.set_config("NM_NT", nt)
            plan = plan_for(M, K, r, c, v, N)
            assert plan.info()["device_kernel"] == "k_nm_mfma", plan.info()
            out[nt] = spmm(plan, B)
            plan.free()
    finally:
        gsa.set_config("NM_NT", old)
    assert np.array_equal(out[0], out[1])
    ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    check(out[1], ref)


@pytest.mark.parametrize("tiles", [2, 4, 7, 8])
@pytest.mark.parametrize("N", [8, 32, 128])
@pytest.mark.parametrize("shape", [(1000, 768), (112 * 3, 512), (1792, 1024), (17, 4096)], ids=lambda s: f"{s[0]}x{s[1]}")
def test_nm_tiles_per_workgroup(shape, N, tiles):
    """k_nm_mfma with 2 / 4 / 7 / 8 sixteen-row tiles per workgroup (NM_TILES; the wave sets
    hold ceil(T/2) and T/2 tiles, the layout one block per set and k-step): row counts that
    end inside a tile, inside a wave set and inside a workgroup, against the oracle"""
    M, K = shape
    r, c, v = thinned(M, K, 40 + M, keep=0.9, empty_rows=(0, M - 1))
    gsa.set_config("NM_TILES", tiles)
    try:
        plan = plan_for(M, K, r, c, v, N)
    finally:
        gsa.set_config("NM_TILES", 0)
    assert plan.info()["device_kernel"] == "k_nm_mfma", plan.info()
    B = np.random.default_rng(M + N).uniform(-1, 1, (K, N)).astype(np.float16)
    ref = ofi.spmm_ref(M, N, r, c, v.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
    assert plan.info()["nm_tiles"] == tiles
    C = spmm(plan, B)
    check(C, ref)

