"""nnz-direction BMTB / BMW blocking and nnz-direction BMTs inside them
(fixed_interval_nnz_direction_{tblock,warp,thread}_blocking_operator.cc with the
get_begin_{rows,nzs}_of_{BMTB,BMW,BMT}_after_fixed_blocking_in_nnz_direction[_relative_to_*],
get_begin_BMWs_of_BMTB_after_blocking, get_begin_BMTs_of_specific_parent_after_blocking,
get_BMW_size_of_each_parent and get_BMTB_size transforms).

- a hand-derived case (BMWs of 4 nonzeros padded, BMTs of 2 inside with relative indices),
- the product vs the oracle restatement, bit-exact, on the canned compositions
  `nnz_warp_bitmap`, `nnz_tblock_bitmap`, `nnz_tblock_warp_bitmap` (token_test.cc:851-870
  runs the BMW + BMT pair; here the thread bitmaps make them executable),
- the validity rules (parent sizes multiples of the child size, relative indices need a
  parent, no padding inside a parent, order of the levels),
- on the GPU (-m gpu): those plans through k_bitmap_segment vs the oracle SpMM."""
import numpy as np
import pytest

import oracle_ffi as ofi

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds
from test_plan_parity import random_coo
from tolerance import bound  # noqa: E402  (contract line + the tight fp16 line)


def test_hand_case():
    """rows 0: cols 0,1,2; row 1: col 3; row 3: cols 0,1 (6 nonzeros, values 1..6).
    BMWs of 4, padded: 8 entries (two copies of (3, 1) with value 0), BMW starts nz
    [0, 4, 8], rows [0, 3, 4], one size 4.  BMTs of 2 inside: nz [0, 2, 4, 6, 8], rows
    [0, 0, 3, 3, 4], relative to their BMW rows [0, 0, 0, 0], nz [0, 2, 0, 2]; the BMWs'
    first BMTs [0, 2, 4]; one BMT size 2."""
    row = np.array([0, 0, 0, 1, 3, 3], np.uint64)
    col = np.array([0, 1, 2, 3, 0, 1], np.uint64)
    val = np.arange(1, 7, dtype=np.float32)
    p = gsa.Plan.from_coo(4, 4, row, col, val)
    p.add_operator("fixed_interval_nnz_direction_warp_blocking_operator", 4, 0, 0, 1)
    p.add_operator("fixed_interval_nnz_direction_thread_blocking_operator", 2, 1, 1, 0)
    a = p.arrays()
    exp = {
        "GLOBAL_META_nz_row_indices_0": [0, 0, 0, 1, 3, 3, 3, 3],
        "GLOBAL_META_nz_col_indices_0": [0, 1, 2, 3, 0, 1, 1, 1],
        "GLOBAL_META_nz_vals_0": [1, 2, 3, 4, 5, 6, 0, 0],
        "WARP_META_first_nz_indices_0": [0, 4, 8],
        "WARP_META_first_row_indices_0": [0, 3, 4],
        "GLOBAL_META_BMW_size_of_each_blk_0": [4],
        "THREAD_META_first_nz_indices_0": [0, 2, 4, 6, 8],
        "THREAD_META_first_row_indices_0": [0, 0, 3, 3, 4],
        "THREAD_META_first_row_indices_relative_to_BMW_0": [0, 0, 0, 0],
        "THREAD_META_first_nz_indices_relative_to_BMW_0": [0, 2, 0, 2],
        "WARP_META_first_BMT_indices_0": [0, 2, 4],
        "GLOBAL_META_BMT_size_of_each_blk_0": [2],
    }
    for k, v in exp.items():
        np.testing.assert_array_equal(a[k].astype(np.float64), np.asarray(v, np.float64), err_msg=k)
    assert p.logical_check() == ""


PIPES = [("nnz_warp_bitmap", 128, 0), ("nnz_warp_bitmap", 32, 0), ("nnz_tblock_bitmap", 256, 0),
         ("nnz_tblock_bitmap", 64, 0), ("nnz_tblock_warp_bitmap", 512, 128), ("nnz_tblock_warp_bitmap", 256, 256)]


def _compare(M, K, r, c, v, name, p0, p1):
    exp, err = ofi.run_pipeline(M, K, r, c, v, name, p0, p1)
    if err is not None:
        with pytest.raises(gsa.GsError):
            gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, 32, p0, p1)
        return None
    p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, 32, p0, p1)
    got = p.arrays()
    assert set(got) == set(exp), (set(got) ^ set(exp))
    for key, arr in exp.items():
        np.testing.assert_array_equal(got[key].astype(np.float64) if arr.dtype == np.float64 else got[key], arr,
                                      err_msg=f"{name}: {key}")
    return p


@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_plans_bit_exact(pipe, seed):
    name, p0, p1 = pipe
    M, K = 150 + 23 * seed, 90
    r, c, v = random_coo(M, K, 0.06 + 0.03 * seed, seed, empty=0.2, trailing_empty=(seed == 1))
    p = _compare(M, K, r, c, v, name, p0, p1)
    assert p is not None
    p.compile()
    assert p.info()["kernel_name"].startswith("k_bitmap_segment")


def test_edge_shapes():
    for M, K, r, c in [(1, 70, np.zeros(70, np.uint64), np.arange(70, dtype=np.uint64)),
                       (70, 1, np.arange(70, dtype=np.uint64), np.zeros(70, np.uint64)),
                       (5, 5, np.array([4], np.uint64), np.array([2], np.uint64))]:
        v = np.linspace(-1, 1, len(r)).astype(np.float32)
        for name, p0, p1 in PIPES:
            _compare(M, K, r, c, v, name, p0, p1)


def test_validity_rules():
    M, K = 60, 50
    r, c, v = random_coo(M, K, 0.2, 4)
    p = gsa.Plan.from_coo(M, K, r, c, v)
    p.add_operator("fixed_interval_nnz_direction_tblock_blocking_operator", 96, 1)
    with pytest.raises(gsa.GsError):  # 96 % 64 != 0 (warp_blocking_operator.cc:60-70)
        p.add_operator("fixed_interval_nnz_direction_warp_blocking_operator", 64, 1, 1, 0)
    with pytest.raises(gsa.GsError):  # padding inside a BMTB (:106-109)
        p.add_operator("fixed_interval_nnz_direction_warp_blocking_operator", 32, 0, 0, 1)
    with pytest.raises(gsa.GsError):  # 96 % 64 != 0 for the BMTs (thread_blocking_operator.cc:66-90)
        p.add_operator("fixed_interval_nnz_direction_thread_blocking_operator", 64, 1, 1, 0)
    p.add_operator("fixed_interval_nnz_direction_warp_blocking_operator", 32, 1, 1, 0)
    p.add_operator("fixed_interval_nnz_direction_thread_blocking_operator", 8, 1, 1, 0)
    assert p.logical_check() == ""
    q = gsa.Plan.from_coo(M, K, r, c, v)
    with pytest.raises(gsa.GsError):  # relative BMW indices without a BMTB
        q.add_operator("fixed_interval_nnz_direction_warp_blocking_operator", 32, 1, 0, 0)
    q.add_operator("fixed_interval_row_direction_tblock_blocking_operator", 4, 0)
    with pytest.raises(gsa.GsError):  # the BMTB level must be the nnz-direction one / first
        q.add_operator("fixed_interval_nnz_direction_tblock_blocking_operator", 64, 1)
    with pytest.raises(gsa.GsError):  # a row-direction parent
        q.add_operator("fixed_interval_nnz_direction_warp_blocking_operator", 32, 0, 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
def test_plans_on_gpu(pipe, dtype):
    torch = pytest.importorskip("torch")
    name, p0, p1 = pipe
    N = 32
    for M, K, row, col, val in [(500, 400, *ds.random_rows(500, 400, 10.0, seed=5, empty_frac=0.2)),
                                (1024, 1024, *ds.rmat(1024, 20000, seed=2))]:
        plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile().upload(dtype, 0)
        assert plan.info()["device_kernel"].startswith("k_bitmap_segment")
        npdt = np.float16 if dtype == "f16" else np.float32
        B = np.random.default_rng(3).uniform(-1, 1, (K, N)).astype(npdt)
        C = plan.spmm(torch.from_numpy(B).to("cuda:0")).float().cpu().numpy()
        v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
        ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
        err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= bound(dtype, plan.info()["device_kernel"]), (name, err.max())
        plan.free()


def test_warp_segment_relative_indices():
    """warp_segment_reduce_operator with relative_row / relative_nz (warp_segment_reduce_operator.cc
    :86-98): the BMTs' row and nz starts relative to their BMW, written next to the absolute
    ones; every relative start = absolute start - its BMW's start, and logical_check holds"""
    r, c, v = ds.random_rows(300, 200, 12.0, seed=1, empty_frac=0.15)
    gsa.set_config("DENSE_MATRIX_SIZE", 32)
    gsa.set_config("VECTOR_WIDTH", 32)
    p = gsa.Plan.from_coo(300, 200, r, c, v)
    p.add_operator("fixed_interval_nnz_direction_thread_blocking_operator", 32, 0, 0, 1)
    p.add_operator("thread_bit_map_operator", 2, 32, 4, 1)
    p.add_operator("warp_segment_reduce_operator", 1, 1, 1)
    a = p.arrays()
    rel_row = a["WARP_META_first_row_indices_relative_to_BMW_0"]
    rel_nz = a["THREAD_META_first_nz_indices_relative_to_BMW_0"]
    fb = a["WARP_META_first_BMT_indices_0"]
    wr, wn = a["WARP_META_first_row_indices_0"], a["WARP_META_first_nz_indices_0"]
    tr, tn = a["THREAD_META_first_row_indices_0"], a["THREAD_META_first_nz_indices_0"]
    for w in range(len(fb) - 1):
        for t in range(int(fb[w]), int(fb[w + 1])):
            assert rel_nz[t] == tn[t] - wn[w]
            if t < len(rel_row):
                assert rel_row[t] == tr[t] - wr[w]
    assert p.logical_check() == ""
