"""Balanced row-direction BMWs (and BMTs: tblock_balanced_thread_total,
balanced_interval_row_direction_thread_blocking_operator.cc:162-249) inside row-direction BMTBs (SURVEY.md §8a A11 inside a parent;
balanced_interval_row_direction_warp_blocking_operator.cc:165-207 with
data_transform_common.cc:794-901): the tblock_balanced_warp_total plans (BMTBs of p0 rows,
BMWs cut after the row whose running count reaches p1 nonzeros, never at a BMTB's last row;
absolute and BMTB-relative indices) bit-exact against the oracle's restatement
(oracle/gs_oracle.c or_balanced_bmw_in_bmtb), a hand case, and the compiled plans on the GPU
against the oracle SpMM."""
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

PIPES = [("tblock_balanced_warp_total", 64, 256), ("tblock_balanced_warp_total", 16, 40),
         ("tblock_balanced_warp_total", 5, 3), ("tblock_balanced_warp_total", 100, 1000),
         ("tblock_balanced_thread_total", 64, 64), ("tblock_balanced_thread_total", 16, 8),
         ("tblock_balanced_thread_total", 7, 3)]


def cases():
    for seed in range(3):
        yield (300 + 11 * seed, 400) + tuple(ds.random_rows(300 + 11 * seed, 400, 9.0, seed=seed, empty_frac=0.15))
    yield (1024, 1024) + tuple(ds.rmat(1024, 20000, seed=2))


@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
def test_plans_bit_exact(pipe):
    name, p0, p1 = pipe
    for M, K, r, c, v in cases():
        exp, err = ofi.run_pipeline(M, K, r, c, v, name, p0, p1)
        assert err is None, err
        p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, 32, p0, p1)
        got = p.arrays()
        assert set(got) == set(exp), set(got) ^ set(exp)
        for key, arr in exp.items():
            np.testing.assert_array_equal(got[key].astype(arr.dtype), arr, err_msg=key)
        assert p.logical_check() == ""
        p.compile()


def test_hand_case():
    """row nnz [2, 0, 3, 1, 5, 0], BMTBs of 4 rows ([0,4) first nz 0, [4,6) first nz 6), 3 nonzeros
    per BMW: BMTB 0 counts 2, 2, 5 -> cut after row 2 (new BMW at row 3, nz 5), row 3 is the
    BMTB's last row; BMTB 1: 5 >= 3 at row 4 -> new BMW at row 5 (nz 11).  Rows [0 3 4 5 6],
    nzs [0 5 6 11 11], relative rows [0 3 0 1], relative nzs [0 5 0 5], first_BMW [0 2 4]."""
    r = np.array([0, 0, 2, 2, 2, 3, 4, 4, 4, 4, 4], np.uint64)
    c = np.array([0, 2, 1, 3, 4, 0, 0, 1, 2, 3, 4], np.uint64)
    v = np.arange(1, 12, dtype=np.float32)
    a = gsa.Plan.from_coo(6, 5, r, c, v).run_pipeline("tblock_balanced_warp_total", 32, 4, 3).arrays()
    assert a["WARP_META_first_row_indices_0"].tolist() == [0, 3, 4, 5, 6]
    assert a["WARP_META_first_nz_indices_0"].tolist() == [0, 5, 6, 11, 11]
    assert a["WARP_META_first_row_indices_relative_to_BMTB_0"].tolist() == [0, 3, 0, 1]
    assert a["WARP_META_first_nz_indices_relative_to_BMTB_0"].tolist() == [0, 5, 0, 5]
    assert a["TBLOCK_META_first_BMW_indices_0"].tolist() == [0, 2, 4]
    exp, err = ofi.run_pipeline(6, 5, r, c, v, "tblock_balanced_warp_total", 4, 3)
    assert err is None and exp["WARP_META_first_row_indices_0"].tolist() == [0, 3, 4, 5, 6]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f16"])
@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}-{p[2]}")
def test_plans_on_gpu(pipe, dtype):
    torch = pytest.importorskip("torch")
    name, p0, p1 = pipe
    for N in (8, 32):
        for M, K, row, col, val in cases():
            plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1)
            plan.compile().upload(dtype, 0)
            npdt = np.float16 if dtype == "f16" else np.float32
            B = np.random.default_rng(3).uniform(-1, 1, (K, N)).astype(npdt)
            C = plan.spmm(torch.from_numpy(B).to("cuda:0")).float().cpu().numpy()
            v = val.astype(np.float16).astype(np.float32) if dtype == "f16" else val
            ref = ofi.spmm_ref(M, N, row, col, v, B.astype(np.float32), "f64")
            err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
            assert err.max() <= bound(dtype, plan.info()["device_kernel"]), (N, plan.info()["device_kernel"], err.max())
            plan.free()
