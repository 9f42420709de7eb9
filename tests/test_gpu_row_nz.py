"""GPU parity of row_nz_matrix_div_operator plans.

The reference's division by row length (operator/row_nz_matrix_div_operator.cc) leaves the
new sub-matrices' row indices in the divided sub-matrix's indexing and can split one row
over two sub-matrices (div_row_indices_by_row_nnz.cc moves on one bucket per entry).  The
executor runs each such sub-matrix into a zeroed scratch output indexed like its parent and
sums the scratch outputs into C (gs::combine_parts), so C must equal the undivided SpMM.
Checked against the oracle's fp64 SpMM with the north-star tolerances (fp32 1e-3, fp16 1e-1
relative to max(1, |ref|)); the sort-based pipelines are not runnable on these sub-matrices
in the reference either (reorder_val_by_index.cc:42 asserts the row count)."""
import numpy as np
import pytest

import oracle_ffi as ofi

torch = pytest.importorskip("torch")
import generalsparse_amd as gsa  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
from tolerance import TOL, bound  # noqa: E402  (contract line + the tight fp16 line, tests/tolerance.py)
# pipelines a row_nz sub-matrix can run (no sort_operator / nnz padding of tiny sub-matrices)
RUNNABLE = [("warp_total", 0, 1), ("block_total", 0, 1), ("tblock_warp_total", 16, 2), ("merge_path", 64, 1),
            ("balanced_warp_total", 64, 1)]


def check(C, ref, dtype, kernel=None):
    """the contract tolerance, and 2^-9 for the fp16 results of fp32-accumulating kernels
    (tests/tolerance.py)"""
    err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
    b = bound(dtype, kernel)
    assert err.max() <= b, f"max rel err {err.max()} > {b} ({kernel})"


def banded(seed, M=120, K=300):
    # bands of similar row length (few division positions: MAX_DIV_TIMES_OF_DIV) + noise rows
    rng = np.random.default_rng(40 + seed)
    lens = np.repeat(rng.choice([0, 3, 12, 40, 90], size=M // 20), 20)
    lens[rng.random(M) < 0.03 * seed] = 1
    rows = np.repeat(np.arange(M, dtype=np.uint64), lens)
    cols = np.concatenate([np.sort(rng.choice(K, size=n, replace=False)) for n in lens]).astype(np.uint64)
    vals = rng.uniform(-1, 1, len(rows)).astype(np.float32)
    return M, K, rows, cols, vals


def spmm(plan, M, K, N, dtype, seed=3):
    npdt = np.float16 if dtype == "f16" else np.float32
    B = np.random.default_rng(seed).uniform(-1, 1, (K, N)).astype(npdt)
    C = torch.full((M, N), float("nan"), dtype=torch.float16 if dtype == "f16" else torch.float32, device=DEV)
    plan.spmm(torch.from_numpy(B).to(DEV), C=C)
    torch.cuda.synchronize()
    Cn = C.float().cpu().numpy()
    assert not np.isnan(Cn).any(), "rows left unwritten"
    return Cn, B


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_straddled_row_hand_case(dtype):
    # rows 0,1 | 2,3 (empty) | 4,5; row 4's first entry lands in sub-matrix 2, its other
    # four in sub-matrix 3 (test_sub_matrix.py::test_row_nz_division_hand_case)
    r = np.repeat(np.array([0, 1, 4, 5], np.uint64), 5)
    c = np.tile(np.arange(5, dtype=np.uint64), 4)
    v = np.arange(1, 21, dtype=np.float32) / 8
    p = gsa.Plan.from_coo(6, 5, r, c, v)
    p.add_operator("row_nz_matrix_div_operator", 4, 64, 2)
    assert p.sub_matrices() == [1, 2, 3]
    for s in p.sub_matrices():
        p.run_pipeline("warp_total", 8, 0, 1, sub=s)
    p.compile().upload(dtype, 0)
    C, B = spmm(p, 6, 5, 8, dtype)
    check(C, ofi.spmm_ref(6, 8, r, c, v, B, "f64"), dtype)


@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("N", [8, 32])
@pytest.mark.parametrize("win,seed", [((4, 64), 0), ((4, 64), 1), ((2, 1024), 0), ((16, 16), 2), ((16, 16), 3),
                                      ((16, 16), 4), ((8, 32), 0), ((3, 512), 1)])
def test_row_nz_plans_match_oracle(win, seed, N, dtype):
    # (window, seed) pairs the operator accepts (at most MAX_DIV_TIMES_OF_DIV positions; the
    # rejection rule itself is tested on the CPU, test_sub_matrix.py)
    M, K, r, c, v = banded(seed)
    p = gsa.Plan.from_coo(M, K, r, c, v)
    p.add_operator("row_nz_matrix_div_operator", win[0], win[1], 2)
    subs = p.sub_matrices()
    assert len(subs) >= 2
    for i, s in enumerate(subs):  # a different kernel family per sub-matrix
        name, p0, p1 = RUNNABLE[(i + seed) % len(RUNNABLE)]
        p.run_pipeline(name, N, p0, p1, sub=s)
    p.compile().upload(dtype, 0)
    C, B = spmm(p, M, K, N, dtype)
    check(C, ofi.spmm_ref(M, N, r, c, v, B, "f64"), dtype)


def test_row_nz_inside_fixed_division():
    # fixed-interval division first (sub-matrices rebased to their own rows), then a row
    # length division of one of them: its sub-matrices refer to rows [120, 240) of C
    M, K, r, c, v = banded(1, M=360)
    N = 8
    p = gsa.Plan.from_coo(M, K, r, c, v)
    subs = p.divide_rows(120)
    assert len(subs) == 3
    p.add_operator("row_nz_matrix_div_operator", 4, 64, 2, sub=subs[1])
    for s in p.sub_matrices():
        p.run_pipeline("merge_path" if s % 2 else "warp_total", N, 64 if s % 2 else 0, 1, sub=s)
    p.compile().upload("f32", 0)
    assert p.info()["n_kernels"] > 3
    C, B = spmm(p, M, K, N, "f32")
    check(C, ofi.spmm_ref(M, N, r, c, v, B, "f64"), "f32")


def test_row_nz_plan_file_computes_the_same(tmp_path):
    M, K, r, c, v = banded(1)
    N = 32
    p = gsa.Plan.from_coo(M, K, r, c, v)
    p.add_operator("row_nz_matrix_div_operator", 4, 64, 2)
    for i, s in enumerate(p.sub_matrices()):
        name, p0, p1 = RUNNABLE[i % len(RUNNABLE)]
        p.run_pipeline(name, N, p0, p1, sub=s)
    p.compile().upload("f16", 0)
    f = tmp_path / "row_nz.gsplan"
    p.save(f)
    q = gsa.Plan.load(f).upload("f16", 0)
    C1, B = spmm(p, M, K, N, "f16")
    C2, _ = spmm(q, M, K, N, "f16")
    assert np.array_equal(C1, C2)
    check(C1, ofi.spmm_ref(M, N, r, c, v, B, "f64"), "f16")


def test_row_nz_replicas_on_two_streams():
    """every plan replica has its own scratch outputs: two replicas launched on
    two streams at once give the single-replica result"""
    M, K, r, c, v = banded(1)
    N = 32
    p = gsa.Plan.from_coo(M, K, r, c, v)
    p.add_operator("row_nz_matrix_div_operator", 4, 64, 2)
    for i, s in enumerate(p.sub_matrices()):
        name, p0, p1 = RUNNABLE[i % len(RUNNABLE)]
        p.run_pipeline(name, N, p0, p1, sub=s)
    p.compile().upload("f32", 0)
    p.add_replica()
    C0, B = spmm(p, M, K, N, "f32")
    Bt = torch.from_numpy(B).to(DEV)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    Ca = torch.empty((M, N), device=DEV)
    Cb = torch.empty((M, N), device=DEV)
    torch.cuda.synchronize()
    for _ in range(20):
        with torch.cuda.stream(s1):
            p.spmm(Bt, C=Ca, replica=0)
        with torch.cuda.stream(s2):
            p.spmm(Bt, C=Cb, replica=1)
    torch.cuda.synchronize()
    assert np.array_equal(Ca.cpu().numpy(), C0) and np.array_equal(Cb.cpu().numpy(), C0)
