"""Row padding to the parent's longest row (modify_{col,vals,row}_*_by_col_pad_parent_blk_to_max_row_size,
SURVEY.md §8a A6/A7 padding branches):
- row-direction BMTs padded to a multiple of a column count inside BMTBs (tblock_thread_total_colpad);
- row padding (modify_*_by_row_pad_in_sub_matrix: the row count up to a multiple of the BMTB /
  BMW height, one zero entry per added row past the matrix) in block_total_rowpad /
  warp_total_rowpad; on the device those plans run into a scratch output of all their rows
  and the first M rows are copied to C;
- row-direction BMTs with is_col_padding_with_row_max_size_with_empty_row, inside BMTBs
  (tblock_thread_total_maxpad) and with no parent (thread_total_maxpad, the ELL-like layout):
  product plan arrays bit-exact against the oracle's restatement (oracle/gs_oracle.c col_pad_max);
- col-direction BMTs after padding without empty rows (tblock/warp_col_thread_maxpad) are in
  test_col_parents.py; the hand-derived cases are in tests/golden/hand_plans.json;
- GPU: the compiled plans against the oracle SpMM."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle_ffi as ofi  # noqa: E402
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402
from tolerance import bound  # noqa: E402  (contract line + the tight fp16 line)

PIPES = [("tblock_thread_total_maxpad", 16, 1), ("tblock_thread_total_maxpad", 4, 2),
         ("tblock_thread_total_maxpad", 3, 3), ("thread_total_maxpad", 1, 0), ("thread_total_maxpad", 4, 0),
         ("tblock_thread_total_colpad", 16, 4), ("tblock_thread_total_colpad", 3, 2),
         ("block_total_rowpad", 16, 0), ("block_total_rowpad", 3, 0), ("warp_total_rowpad", 16, 0),
         ("warp_total_rowpad", 5, 0)]


def cases():
    for seed in range(3):
        yield ("rows", 200, 300) + tuple(ds.random_rows(200, 300, 12.0, seed=seed, empty_frac=0.1))
    r = np.array([0, 0, 2, 2, 2, 3, 4, 4, 4, 4, 4], np.uint64)
    c = np.array([0, 2, 1, 3, 4, 0, 0, 1, 2, 3, 4], np.uint64)
    yield ("ex1_like", 7, 5, r, c, np.linspace(-1, 1, len(r)).astype(np.float32))  # trailing empty rows


@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
def test_plans_bit_exact(pipe):
    name, p0, p1 = pipe
    for _, M, K, r, c, v in cases():
        exp, err = ofi.run_pipeline(M, K, r, c, v, name, p0, p1)
        assert err is None, err
        p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, 32, p0, p1)
        got = p.arrays()
        assert set(got) == set(exp), set(got) ^ set(exp)
        for key, arr in exp.items():
            np.testing.assert_array_equal(got[key].astype(arr.dtype), arr, err_msg=f"{name}: {key}")
        assert p.logical_check() == ""
        p.compile()


def test_padding_rate_bound():
    # one row of 60 among rows of 1: padding every row to 60 is >= PADDING_RATE_UP_BOUND (4)
    r = np.concatenate([np.zeros(60, np.uint64), np.arange(1, 40, dtype=np.uint64)])
    c = np.concatenate([np.arange(60, dtype=np.uint64), np.zeros(39, np.uint64)])
    v = np.ones(len(r), np.float32)
    exp, err = ofi.run_pipeline(40, 60, r, c, v, "thread_total_maxpad", 1, 0)
    assert exp is None and err
    with pytest.raises(gsa.GsError):
        gsa.Plan.from_coo(40, 60, r, c, v).run_pipeline("thread_total_maxpad", 32, 1, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
def test_plans_on_gpu(pipe, dtype):
    torch = pytest.importorskip("torch")
    name, p0, p1 = pipe
    for N in (8, 32):
        for _, M, K, row, col, val in cases():
            plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile().upload(dtype, 0)
            npdt = np.float16 if dtype == "f16" else np.float32
            B = np.random.default_rng(3).uniform(-1, 1, (K, N)).astype(npdt)
            C = plan.spmm(torch.from_numpy(B).to("cuda:0")).float().cpu().numpy()
            v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
            ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
            err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
            assert err.max() <= bound(dtype, plan.info()["device_kernel"]), (name, N, plan.info()["device_kernel"], err.max())
            plan.free()


def test_row_pad_hand_case():
    """ex1-like 7 x 5 matrix, BMTBs of 4 rows with row padding: end_row_index 6 -> 7 rows, one
    row added (row 7, the last column 4, value 0); BMTB rows [0, 4, 8], first nz [0, 6, 12]"""
    r = np.array([0, 0, 2, 2, 2, 3, 4, 4, 4, 4, 4], np.uint64)
    c = np.array([0, 2, 1, 3, 4, 0, 0, 1, 2, 3, 4], np.uint64)
    v = np.arange(1, 12, dtype=np.float32)
    a = gsa.Plan.from_coo(7, 5, r, c, v).run_pipeline("block_total_rowpad", 32, 4, 0).arrays()
    assert a["GLOBAL_META_nz_row_indices_0"].tolist() == [0, 0, 2, 2, 2, 3, 4, 4, 4, 4, 4, 7]
    assert a["GLOBAL_META_nz_col_indices_0"].tolist() == [0, 2, 1, 3, 4, 0, 0, 1, 2, 3, 4, 4]
    assert a["GLOBAL_META_nz_vals_0"].tolist() == list(range(1, 12)) + [0]
    assert a["TBLOCK_META_first_row_indices_0"].tolist() == [0, 4, 8]
    assert a["TBLOCK_META_first_nz_indices_0"].tolist() == [0, 6, 12]
