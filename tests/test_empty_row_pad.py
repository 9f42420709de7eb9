"""empty_row_pad_operator (operator/empty_row_pad_operator.cc, with
modify_{col,val,row}_*_by_empty_pad_in_submatrix.cc): every empty row between the first
nonzero and the end of the sub-matrix gets one zero entry.

- a hand-derived case (worked from the cited transforms, including the leading empty row the
  reference's walk never reaches),
- the product vs the oracle restatement, bit-exact, alone and followed by the canned
  pipelines (`empty_pad_<pipeline>`),
- the operator's validity rules (not after sort_operator, not twice, not after blocking,
  needs an empty row),
- on the GPU (-m gpu): the padded plans through their kernels vs the oracle SpMM."""
import numpy as np
import pytest

import oracle_ffi as ofi

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds
from test_plan_parity import oracle_params, random_coo
from tolerance import bound  # noqa: E402  (contract line + the tight fp16 line)

G = "GLOBAL_META_"


def test_hand_case():
    """rows 0..6, nonzeros (1,2) (1,4) (3,0) (4,5) with values 1..4:
    row 1 is followed by row 3 -> one entry for row 2 (column 4, value 0); the last nonzero
    (row 4) is followed by the row count 7 -> entries for rows 5 and 6 (column 5); row 0
    precedes the first nonzero and stays empty"""
    row = np.array([1, 1, 3, 4], np.uint64)
    col = np.array([2, 4, 0, 5], np.uint64)
    val = np.array([1, 2, 3, 4], np.float32)
    p = gsa.Plan.from_coo(7, 6, row, col, val)
    p.add_operator("empty_row_pad_operator")
    a = p.arrays()
    np.testing.assert_array_equal(a[G + "nz_row_indices_0"], [1, 1, 2, 3, 4, 5, 6])
    np.testing.assert_array_equal(a[G + "nz_col_indices_0"], [2, 4, 4, 0, 5, 5, 5])
    np.testing.assert_array_equal(a[G + "nz_vals_0"], [1, 2, 0, 3, 4, 0, 0])
    exp, err = ofi.run_pipeline(7, 6, row, col, val, "empty_row_pad")
    assert err is None
    for k in ("nz_row_indices_0", "nz_col_indices_0", "nz_vals_0"):
        np.testing.assert_array_equal(a[G + k].astype(exp[G + k].dtype), exp[G + k])
    assert "empty_row_pad_operator" in p.log()


def _compare(M, K, r, c, v, inner, N, p0, p1):
    name = "empty_pad_" + inner
    exp, err = ofi.run_pipeline(M, K, r, c, v, name, oracle_params(inner, N, p0, p1),
                                p1 if inner in ("merge_path", "tblock_warp_total_relative", "tblock_warp_total") else 0)
    if err is not None:
        with pytest.raises(gsa.GsError):
            gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, N, p0, p1)
        return None
    p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, N, p0, p1)
    got = p.arrays()
    for key, arr in exp.items():
        assert key in got, f"{name}: product lacks {key}"
        np.testing.assert_array_equal(got[key].astype(np.float64) if arr.dtype == np.float64 else got[key], arr,
                                      err_msg=f"{name}: {key}")
    return p


INNER = [("warp_total", 32, 0, 1), ("block_total", 8, 4, 1), ("tblock_warp_total", 32, 20, 2),
         ("thread_bit_map", 32, 4, 1), ("warp_segment", 32, 4, 1), ("balanced_warp_total", 32, 64, 1),
         ("merge_path", 8, 16, 1), ("tblock_thread_total", 32, 16, 1)]


@pytest.mark.parametrize("pipe", INNER, ids=lambda p: p[0])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_padded_pipelines_bit_exact(pipe, seed):
    inner, N, p0, p1 = pipe
    M, K = 120 + 17 * seed, 90
    r, c, v = random_coo(M, K, 0.08, seed, empty=0.3, trailing_empty=(seed == 1))
    p = _compare(M, K, r, c, v, inner, N, p0, p1)
    assert p is not None
    p.compile()
    # every row from the first nonzero row on holds an entry now
    rows = p.arrays()[G + "nz_row_indices_0"]
    assert set(range(int(rows.min()), M)) <= set(rows.tolist())


def test_validity_rules():
    M, K = 40, 30
    r, c, v = random_coo(M, K, 0.2, 3, empty=0.3)
    p = gsa.Plan.from_coo(M, K, r, c, v)
    p.add_operator("sort_operator")
    with pytest.raises(gsa.GsError):  # after sort_operator (empty_row_pad_operator.cc:37-52)
        p.add_operator("empty_row_pad_operator")
    q = gsa.Plan.from_coo(M, K, r, c, v)
    q.add_operator("empty_row_pad_operator")
    with pytest.raises(gsa.GsError):  # twice
        q.add_operator("empty_row_pad_operator")
    b = gsa.Plan.from_coo(M, K, r, c, v)
    b.add_operator("fixed_interval_row_direction_tblock_blocking_operator", 4, 0)
    with pytest.raises(gsa.GsError):  # after a distributing operator
        b.add_operator("empty_row_pad_operator")
    full_r = np.repeat(np.arange(M, dtype=np.uint64), 2)
    full_c = np.tile(np.array([0, 1], np.uint64), M)
    f = gsa.Plan.from_coo(M, K, full_r, full_c, np.ones(2 * M, np.float32))
    with pytest.raises(gsa.GsError):  # no empty row (:124)
        f.add_operator("empty_row_pad_operator")
    # one nonzero among 40 rows: 39 padding entries, rate 40 >= PADDING_RATE_UP_BOUND (4)
    s = gsa.Plan.from_coo(M, K, np.array([0], np.uint64), np.array([0], np.uint64), np.ones(1, np.float32))
    with pytest.raises(gsa.GsError):
        s.add_operator("empty_row_pad_operator")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", INNER, ids=lambda p: p[0])
def test_padded_plans_on_gpu(pipe, dtype):
    torch = pytest.importorskip("torch")
    inner, _, p0, p1 = pipe
    N = 32
    M, K = 500, 400
    row, col, val = ds.random_rows(M, K, 10.0, seed=21, empty_frac=0.25)
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("empty_pad_" + inner, N, p0, p1).compile()
    plan.upload(dtype, 0)
    npdt = np.float16 if dtype == "f16" else np.float32
    B = np.random.default_rng(2).uniform(-1, 1, (K, N)).astype(npdt)
    C = plan.spmm(torch.from_numpy(B).to("cuda:0")).float().cpu().numpy()
    v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
    ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
    err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= bound(dtype, plan.info()["device_kernel"]), (inner, err.max())
    plan.free()
