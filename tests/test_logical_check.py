"""logical_check (metadata_set.cc:806-1890): every pipeline's plan is consistent, and a
corrupted plan array is caught -- by gs_plan_logical_check and by gs_plan_compile, which
runs it as token_test asserts it after every pipeline (token_test.cc:517-1541)."""
import numpy as np
import pytest

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds

PIPES = [("thread_total", 4, 1), ("warp_total", 0, 1), ("block_total", 20, 1), ("thread_bit_map", 4, 1),
         ("warp_segment", 4, 1), ("tblock_warp_total", 20, 2), ("balanced_warp_total", 256, 1),
         ("col_direction_nm", 32, 1), ("merge_path", 64, 1), ("merge_path", 7, 3), ("merge_path", 4096, 2),
         ("balanced_block_total", 512, 1), ("balanced_thread_total", 64, 1), ("tblock_thread_total", 16, 1),
         ("tblock_warp_thread_total", 16, 2), ("tblock_warp_total_relative", 16, 2)]


def matrices():
    yield 300, 200, ds.random_rows(300, 200, 12.0, seed=1)
    yield 1024, 1024, ds.rmat(1024, 20000, seed=2)
    yield 256, 512, ds.pruned_weight(256, 512, 0.7, 13)
    yield 64, 256, ds.two_four(64, 256, 3)


@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-{p[1]}")
def test_every_pipeline_is_consistent(pipe):
    for M, K, (r, c, v) in matrices():
        try:
            plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(pipe[0], 32, pipe[1], pipe[2])
        except gsa.GsError:
            continue  # the operator's validity rules refuse this matrix (e.g. col-direction on ragged rows)
        assert plan.logical_check() == "", (pipe, M)
        plan.compile()


def test_divided_plan_is_consistent():
    r, c, v = ds.random_rows(600, 300, 9.0, seed=3, empty_frac=0.1)
    plan = gsa.Plan.from_coo(600, 300, r, c, v)
    subs = plan.divide_rows(200)
    for s in subs:
        plan.run_pipeline("tblock_warp_total", 32, 16, 2, sub=s)
    assert plan.logical_check() == ""
    plan.compile()


# (pipeline, p0, p1, array to corrupt, index, delta, words of the expected violation)
CORRUPT = [
    ("thread_total", 4, 1, "THREAD_META_first_nz_indices_0", 7, 4, "disagree with the rows"),
    ("block_total", 20, 1, "TBLOCK_META_first_nz_indices_0", 0, 1, "start at 0"),
    ("block_total", 20, 1, "TBLOCK_META_first_nz_indices_0", -1, 1, "stored nnz"),
    ("tblock_warp_total", 20, 2, "TBLOCK_META_first_BMW_indices_0", 2, 1, "first_BMW_indices"),
    ("warp_segment", 4, 1, "WARP_META_first_BMT_indices_0", 1, 1, "first_BMT_indices"),
    ("tblock_thread_total", 16, 1, "THREAD_META_first_nz_indices_relative_to_BMTB_0", 5, 1, "relative_to_BMTB"),
    ("tblock_warp_thread_total", 16, 2, "THREAD_META_first_row_indices_relative_to_BMW_0", 3, 1, "relative_to_BMW"),
    ("tblock_warp_total_relative", 16, 2, "WARP_META_first_nz_indices_relative_to_BMTB_0", 3, 2, "relative_to_BMTB"),
    ("col_direction_nm", 32, 1, "THREAD_META_first_row_indices_without_ending_0", 3, 1, "without_ending"),
    ("thread_total", 4, 1, "GLOBAL_META_nz_row_indices_0", 5, 200, "not sorted"),
    ("warp_total", 0, 1, "GLOBAL_META_nz_col_indices_0", 9, 10 ** 6, "columns"),
]


@pytest.mark.parametrize("case", CORRUPT, ids=lambda c: f"{c[0]}-{c[3].split('META_')[1]}")
def test_corrupted_plan_is_refused(case):
    name, p0, p1, key, idx, delta, words = case
    r, c, v = ds.pruned_weight(256, 512, 0.7, 13) if name == "col_direction_nm" or "tblock" in name \
        else ds.random_rows(300, 200, 12.0, seed=1)
    M, K = (256, 512) if name == "col_direction_nm" or "tblock" in name else (300, 200)
    if name == "col_direction_nm":
        r, c, v = ds.two_four(64, 256, 3)
        M, K = 64, 256
    plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline(name, 32, p0, p1)
    assert plan.logical_check() == ""
    a = plan.array(key)
    i = idx % len(a)
    plan.set_array_entry(key, i, int(a[i]) + delta)
    msg = plan.logical_check()
    assert words in msg, msg
    with pytest.raises(gsa.GsError, match="logical_check"):
        plan.compile()


def test_merged_col_direction_rows_one_short_are_accepted():
    """929 col-direction BMTs merged 32 to a BMW: get_begin_rows_after_merge_thread.cc:39-44
    leaves the BMW row starts one short of the nz starts (30 vs 31) when n_BMT - 1 is a
    multiple of 32; the plan runs (its kernel reads the BMT arrays) and is accepted, the
    short array checked as group starts without an ending"""
    row, col, _ = ds.random_rows(200, 1500, 300.0, seed=9, empty_frac=0.1)
    p = gsa.Plan.from_coo(200, 1500, row, col, np.ones(len(row), np.float32)).run_pipeline("warp_bit_map", 32, 4, 1)
    a = p.arrays()
    assert len(a["THREAD_META_first_nz_indices_0"]) == 930
    assert len(a["WARP_META_first_row_indices_0"]) + 1 == len(a["WARP_META_first_nz_indices_0"]) == 31
    p.compile()
    assert p.logical_check() == ""
    # still a real check: a decreasing group start is caught
    p.set_array_entry("WARP_META_first_row_indices_0", 5, 0)
    assert "decreasing" in p.logical_check()
