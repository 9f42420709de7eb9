"""col-direction BMWs / BMTBs and col-direction BMTs inside row-direction parents
(fixed_interval_col_direction_{tblock,warp,thread}_blocking_operator.cc with the
get_begin_{rows,nzs}_of_{BMTB,BMW}_after_fixed_blocking_in_col_direction[_relative_to_BMTB],
get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_{BMTB,BMW},
get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents,
get_begin_{BMWs,BMTs}_of_..._after_blocking, get_BMT_size_of_each_parent and
remove_item_of_metadata transforms; the padded BMT blocking re-runs the former operators).

- a hand-derived case (BMTs of 2 nonzeros inside BMTBs of 2 rows, relative indices),
- the product vs the oracle restatement, bit-exact, on the canned compositions,
- the validity rules (first distributing operator for the col BMTB level, no col level after
  a col level, relative indices need a parent),
- on the GPU (-m gpu): the plans through k_row_chunks (the chunk level named by the plan) vs
  the oracle SpMM."""
import numpy as np
import pytest

import oracle_ffi as ofi

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds
from test_plan_parity import random_coo
from tolerance import bound  # noqa: E402  (contract line + the tight fp16 line)


def test_hand_case():
    """rows 0: cols 0,1,2; row 1: col 3; row 2: empty; row 3: cols 0,1,2,3,4 (9 nonzeros).
    BMTBs of 2 rows: rows [0, 2, 4], nz [0, 4, 9].  BMTs of 2 nonzeros: rows (no ending)
    [0, 0, 1, 3, 3, 3], nz [0, 2, 3, 4, 6, 8, 9]; relative to the BMTB rows [0, 0, 1, 1, 1, 1],
    nz [0, 2, 3, 0, 2, 4]; the BMTBs' first BMTs [0, 3, 6]."""
    row = np.array([0, 0, 0, 1, 3, 3, 3, 3, 3], np.uint64)
    col = np.array([0, 1, 2, 3, 0, 1, 2, 3, 4], np.uint64)
    val = np.arange(1, 10, dtype=np.float32)
    p = gsa.Plan.from_coo(4, 5, row, col, val)
    p.add_operator("fixed_interval_row_direction_tblock_blocking_operator", 2, 0)
    p.add_operator("fixed_interval_col_direction_thread_blocking_operator", 2, 1, 1, 0, 0)
    a = p.arrays()
    exp = {
        "TBLOCK_META_first_row_indices_0": [0, 2, 4],
        "TBLOCK_META_first_nz_indices_0": [0, 4, 9],
        "THREAD_META_first_row_indices_without_ending_0": [0, 0, 1, 3, 3, 3],
        "THREAD_META_first_nz_indices_0": [0, 2, 3, 4, 6, 8, 9],
        "THREAD_META_first_row_indices_relative_to_BMTB_0": [0, 0, 1, 1, 1, 1],
        "THREAD_META_first_nz_indices_relative_to_BMTB_0": [0, 2, 3, 0, 2, 4],
        "TBLOCK_META_first_BMT_indices_0": [0, 3, 6],
    }
    for k, v in exp.items():
        np.testing.assert_array_equal(a[k].astype(np.float64), np.asarray(v, np.float64), err_msg=k)
    assert p.logical_check() == ""


def test_hand_case_col_warp_and_padding():
    """The same matrix.  col-direction BMWs of 3: rows [0, 1, 3, 3], nz [0, 3, 4, 7, 9].
    Padded BMTs of 2 inside BMTBs of 2 rows: rows padded to 4, 2, 0, 6 entries (pad = the
    row's last column, value 0), the BMTBs rebuilt on the padded COO (nz [0, 6, 12]), BMTs
    nz [0, 2, 4, 6, 8, 10, 12], per-BMTB BMT size [2, 2], one global size 2."""
    row = np.array([0, 0, 0, 1, 3, 3, 3, 3, 3], np.uint64)
    col = np.array([0, 1, 2, 3, 0, 1, 2, 3, 4], np.uint64)
    val = np.arange(1, 10, dtype=np.float32)
    p = gsa.Plan.from_coo(4, 5, row, col, val)
    p.add_operator("fixed_interval_col_direction_warp_blocking_operator", 3, 0, 0, 0, 0)
    a = p.arrays()
    assert a["WARP_META_first_row_indices_without_ending_0"].tolist() == [0, 1, 3, 3]
    assert a["WARP_META_first_nz_indices_0"].tolist() == [0, 3, 4, 7, 9]
    q = gsa.Plan.from_coo(4, 5, row, col, val)
    q.add_operator("fixed_interval_row_direction_tblock_blocking_operator", 2, 0)
    q.add_operator("fixed_interval_col_direction_thread_blocking_operator", 2, 1, 1, 1, 0)
    b = q.arrays()
    assert b["GLOBAL_META_nz_row_indices_0"].tolist() == [0, 0, 0, 0, 1, 1, 3, 3, 3, 3, 3, 3]
    assert b["GLOBAL_META_nz_col_indices_0"].tolist() == [0, 1, 2, 2, 3, 3, 0, 1, 2, 3, 4, 4]
    assert b["GLOBAL_META_nz_vals_0"].tolist() == [1, 2, 3, 0, 4, 0, 5, 6, 7, 8, 9, 0]
    assert b["TBLOCK_META_first_nz_indices_0"].tolist() == [0, 6, 12]
    assert b["THREAD_META_first_nz_indices_0"].tolist() == [0, 2, 4, 6, 8, 10, 12]
    assert b["TBLOCK_META_BMT_size_of_each_blk_0"].tolist() == [2, 2]
    assert b["GLOBAL_META_BMT_size_of_each_blk_0"].tolist() == [2]
    assert q.logical_check() == ""


PIPES = [("col_warp_total", 16, 0), ("col_warp_total", 5, 0), ("col_tblock_total", 40, 0),
         ("tblock_col_warp_total", 16, 8), ("tblock_col_warp_total", 7, 3), ("tblock_col_thread_total", 16, 8),
         ("tblock_col_thread_total", 5, 4), ("warp_col_thread_total", 4, 8), ("warp_col_thread_total", 1, 3),
         ("tblock_col_thread_total_padded", 16, 8), ("tblock_col_thread_total_padded", 3, 4),
         ("tblock_col_thread_interleaved", 16, 8), ("tblock_col_thread_interleaved", 3, 4),
         ("warp_col_thread_interleaved", 8, 8), ("warp_col_thread_interleaved", 1, 4),
         ("tblock_col_thread_maxpad", 16, 8), ("tblock_col_thread_maxpad", 3, 4),
         ("warp_col_thread_maxpad", 8, 8), ("warp_col_thread_maxpad", 1, 2)]


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
    assert p.info()["kernel_name"].startswith("k_row_chunks")


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
    p.add_operator("fixed_interval_row_direction_tblock_blocking_operator", 4, 0)
    with pytest.raises(gsa.GsError):  # the col-direction BMTB level is the first distributing one
        p.add_operator("fixed_interval_col_direction_tblock_blocking_operator", 16, 0, 0)
    p.add_operator("fixed_interval_col_direction_warp_blocking_operator", 16, 1, 1, 0, 0)
    with pytest.raises(gsa.GsError):  # no col-direction BMTs after a col-direction level
        p.add_operator("fixed_interval_col_direction_thread_blocking_operator", 4, 1, 1, 0, 0)
    q = gsa.Plan.from_coo(M, K, r, c, v)
    with pytest.raises(gsa.GsError):  # relative BMW indices without a BMTB
        q.add_operator("fixed_interval_col_direction_warp_blocking_operator", 16, 1, 0, 0, 0)
    # padding to the parent's max row size at GLOBAL level (no parent): every non-empty row to
    # the longest row, then col-direction BMWs of 16
    q.add_operator("fixed_interval_col_direction_warp_blocking_operator", 16, 0, 0, 0, 1)
    a = q.arrays()
    cnt = np.bincount(a["GLOBAL_META_nz_row_indices_0"].astype(np.int64), minlength=M)
    assert set(cnt[cnt > 0].tolist()) == {np.bincount(r.astype(np.int64)).max()}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
def test_plans_on_gpu(pipe, dtype):
    torch = pytest.importorskip("torch")
    name, p0, p1 = pipe
    for N in (8, 32):
        for M, K, row, col, val in [(500, 400, *ds.random_rows(500, 400, 10.0, seed=5, empty_frac=0.2)),
                                    (1024, 1024, *ds.rmat(1024, 20000, seed=2))]:
            plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile().upload(dtype, 0)
            assert plan.info()["device_kernel"].startswith("k_row_chunks")
            npdt = np.float16 if dtype == "f16" else np.float32
            B = np.random.default_rng(3).uniform(-1, 1, (K, N)).astype(npdt)
            C = plan.spmm(torch.from_numpy(B).to("cuda:0")).float().cpu().numpy()
            v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
            ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
            err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
            assert err.max() <= bound(dtype, plan.info()["device_kernel"]), (name, N, err.max())
            plan.free()


def test_interleaved_in_tblock_parent_plan_file(tmp_path):
    """per-BMTB interleaved storage: the compiled spec names the parent, and a plan file keeps
    it (GSPLAN03 stores 2 + parent level in the interleave field)"""
    M, K = 120, 70
    r, c, v = random_coo(M, K, 0.1, 7, empty=0.2)
    p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("tblock_col_thread_interleaved", 32, 8, 4).compile()
    assert p.info()["kernel_name"] == "k_row_chunks+interleaved"
    f = str(tmp_path / "ilv.gsplan")
    p.save(f)
    q = gsa.Plan.load(f)
    assert q.info()["kernel_name"] == "k_row_chunks+interleaved"
    a, b = p.arrays(), q.arrays()
    for k in ("GLOBAL_META_nz_col_indices_after_interlance_storage_0", "TBLOCK_META_first_BMT_indices_0"):
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_interleaved_in_tblock_parent_loaded_plan_on_gpu(tmp_path, dtype):
    """the per-BMTB interleaved plan, saved and loaded, computes the same C on the device"""
    torch = pytest.importorskip("torch")
    M, K, N = 700, 300, 32
    row, col, val = ds.random_rows(M, K, 12.0, seed=9, empty_frac=0.1)
    p = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("tblock_col_thread_interleaved", N, 16, 8).compile()
    f = str(tmp_path / "ilv.gsplan")
    p.save(f)
    npdt = np.float16 if dtype == "f16" else np.float32
    B = torch.from_numpy(np.random.default_rng(4).uniform(-1, 1, (K, N)).astype(npdt)).to("cuda:0")
    Cs = []
    for plan in (p.upload(dtype, 0), gsa.Plan.load(f).upload(dtype, 0)):
        assert plan.info()["device_kernel"].startswith("k_row_chunks")
        Cs.append(plan.spmm(B).float().cpu().numpy())
        plan.free()
    v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
    ref = ofi.spmm_ref(M, N, row, col, v, B.float().cpu().numpy(), "f64")
    for C in Cs:
        err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= bound(dtype, "k_row_chunks"), err.max()
