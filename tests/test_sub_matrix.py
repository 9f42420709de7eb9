"""Sub-matrix splits, CPU part.

fixed_interval_row_matrix_div_operator (operator/fixed_interval_row_matrix_div_operator.cc)
splits a sub-matrix into one new sub-matrix per non-empty interval of
fixed_row_interval_size rows; each new sub-matrix then gets its own operators and its own
kernel.  Checked here:
  - the division's arrays are bit-identical to the oracle's restatement
    (or_fixed_interval_row_div) and to a hand-derived case;
  - a pipeline run on sub-matrix s produces exactly the arrays the oracle produces for a
    standalone matrix holding that sub-matrix's rows (the transforms work on rows relative
    to the sub-matrix, so the two agree key for key apart from the sub-matrix suffix);
  - the operator's validity rules (:30-150): no second division of the same target, more
    rows than the interval, at most MAX_DIV_TIMES_OF_DIV intervals, none after
    interleaved storage.
"""
import numpy as np
import pytest

import oracle_ffi as ofi

import generalsparse_amd as gsa
from test_plan_parity import oracle_params, random_coo

BOUNDARY = ("begin_row_index", "end_row_index", "begin_col_index", "end_col_index")


def divided(M, K, r, c, v, gap):
    p = gsa.Plan.from_coo(M, K, r, c, v)
    return p, p.divide_rows(gap)


def check_division(M, K, r, c, v, gap):
    exp, err = ofi.run_pipeline(M, K, r, c, v, "row_div", gap, 0)
    if err is not None:
        with pytest.raises(gsa.GsError):
            divided(M, K, r, c, v, gap)
        return None, None
    p, subs = divided(M, K, r, c, v, gap)
    got = p.arrays()
    assert sorted(got) == sorted(exp)
    for k, a in exp.items():
        np.testing.assert_array_equal(got[k], a, err_msg=k)
    assert subs == sorted({int(k.rsplit("_", 1)[1]) for k in exp if "nz_col_indices" in k})
    return p, subs


def test_division_hand_case():
    # rows 0,0,1 | (3..5 empty) | 6,6 with gap 3: intervals 0 and 2 are non-empty
    r = np.array([0, 0, 1, 6, 6], np.uint64)
    c = np.array([1, 4, 2, 0, 3], np.uint64)
    v = np.arange(1, 6, dtype=np.float32)
    p, subs = check_division(7, 5, r, c, v, 3)
    assert subs == [1, 2]
    a = p.arrays()
    assert a["GLOBAL_META_begin_row_index_1"].tolist() == [0] and a["GLOBAL_META_end_row_index_1"].tolist() == [2]
    assert a["GLOBAL_META_begin_row_index_2"].tolist() == [6] and a["GLOBAL_META_end_row_index_2"].tolist() == [6]
    assert a["GLOBAL_META_nz_row_indices_1"].tolist() == [0, 0, 1]
    assert a["GLOBAL_META_nz_row_indices_2"].tolist() == [0, 0]
    assert a["GLOBAL_META_nz_col_indices_2"].tolist() == [0, 3]
    assert a["GLOBAL_META_nz_vals_2"].tolist() == [4.0, 5.0]
    assert a["GLOBAL_META_end_col_index_1"].tolist() == [4]
    assert "GLOBAL_META_nz_row_indices_0" not in a and "GLOBAL_META_begin_row_index_0" in a


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("gap", [7, 32, 50, 64, 100])
def test_division_matches_oracle(seed, gap):
    M, K = 300 + 17 * seed, 120
    r, c, v = random_coo(M, K, 0.05, seed, empty=0.3, trailing_empty=seed % 2 == 1)
    if seed == 3:  # a band of empty rows: an empty interval in the middle
        keep = (r < 90) | (r >= 210)
        r, c, v = r[keep], c[keep], v[keep]
    check_division(M, K, r, c, v, gap)


def test_division_validity():
    r, c, v = random_coo(200, 60, 0.1, 5, empty=0.0)
    p = gsa.Plan.from_coo(200, 60, r, c, v)
    with pytest.raises(gsa.GsError):  # no more rows than the interval
        p.add_operator("fixed_interval_row_matrix_div_operator", 200)
    with pytest.raises(gsa.GsError):  # 20 intervals > MAX_DIV_TIMES_OF_DIV (12)
        p.add_operator("fixed_interval_row_matrix_div_operator", 10)
    subs = p.divide_rows(50)
    assert subs == [1, 2, 3, 4]
    with pytest.raises(gsa.GsError):  # sub-matrix 0 was divided already
        p.add_operator("fixed_interval_row_matrix_div_operator", 60)
    # a new sub-matrix can be divided again (nested division, ids continue from the max)
    assert p.divide_rows(20, sub=2) == [1, 3, 4, 5, 6, 7]
    a = p.arrays()
    assert a["GLOBAL_META_begin_row_index_5"].tolist() == [50]
    assert a["GLOBAL_META_end_row_index_7"].tolist() == [99]


def test_division_after_interleaving_rejected():
    r, c, v = random_coo(128, 512, 0.3, 1, empty=0.0)
    p = gsa.Plan.from_coo(128, 512, r, c, v)
    p.run_pipeline("warp_bit_map_interleaved", 32, 4, 1)
    with pytest.raises(gsa.GsError):
        p.add_operator("fixed_interval_row_matrix_div_operator", 32)


SUB_PIPES = [("thread_total", 32, 4, 1), ("warp_total", 32, 0, 1), ("block_total", 8, 0, 1),
             ("thread_bit_map", 32, 4, 1), ("warp_segment", 32, 4, 1), ("tblock_warp_total", 32, 4, 1),
             ("balanced_warp_total", 32, 64, 1), ("balanced_block_total", 32, 64, 1),
             ("balanced_thread_total", 8, 16, 1), ("merge_path", 8, 16, 1), ("merge_path", 32, 5, 3),
             ("tblock_warp_total_relative", 32, 20, 2)]


def sub_coo(p, s):
    a = p.arrays()
    rows = int(a[f"GLOBAL_META_end_row_index_{s}"][0] - a[f"GLOBAL_META_begin_row_index_{s}"][0] + 1)
    return (rows, a[f"GLOBAL_META_nz_row_indices_{s}"], a[f"GLOBAL_META_nz_col_indices_{s}"],
            a[f"GLOBAL_META_nz_vals_{s}"].astype(np.float32))


@pytest.mark.parametrize("pipe", SUB_PIPES, ids=lambda p: f"{p[0]}-N{p[1]}-{p[2]}-{p[3]}")
@pytest.mark.parametrize("seed", [0, 1])
def test_sub_matrix_plans_match_standalone_oracle(pipe, seed):
    name, N, p0, p1 = pipe
    M, K = 260 + 40 * seed, 150
    r, c, v = random_coo(M, K, 0.06, 10 + seed, empty=0.25, trailing_empty=True)
    keep = (r < 60) | (r >= 130)
    r, c, v = r[keep], c[keep], v[keep]
    p, subs = divided(M, K, r, c, v, 64)
    planned = 0
    for s in subs:
        rows, sr, sc, sv = sub_coo(p, s)
        exp, err = ofi.run_pipeline(rows, K, sr, sc, sv, name, oracle_params(name, N, p0, p1),
                                    p1 if name in ("merge_path", "tblock_warp_total_relative") else 0)
        if err is not None:
            with pytest.raises(gsa.GsError):
                p.run_pipeline(name, N, p0, p1, sub=s)
            continue
        p.run_pipeline(name, N, p0, p1, sub=s)
        planned += 1
        got = p.arrays()
        for k, arr in exp.items():
            pos_name, sub = k.rsplit("_", 1)
            if sub == "-1" or any(pos_name.endswith(b) for b in BOUNDARY):
                continue
            gk = f"{pos_name}_{s}"
            assert gk in got, f"{name}: sub-matrix {s} lacks {gk}"
            np.testing.assert_array_equal(got[gk], arr, err_msg=f"{name} sub {s}: {gk}")
    if planned < len(subs):
        return
    p.compile()
    info = p.info()
    assert info["n_kernels"] == len(subs)
    assert info["nnz_stored"] >= len(r)


def test_compile_needs_every_sub_matrix():
    r, c, v = random_coo(200, 60, 0.1, 6, empty=0.0)
    p = gsa.Plan.from_coo(200, 60, r, c, v)
    subs = p.divide_rows(64)
    p.run_pipeline("warp_total", 32, 0, 1, sub=subs[0])
    with pytest.raises(gsa.GsError):
        p.compile()
    for s in subs[1:]:
        p.run_pipeline("thread_total", 32, 4, 1, sub=s)
    p.compile()
    with pytest.raises(gsa.GsError):  # emitted programs hold one kernel
        p.generate_program("/tmp/gs_never_written")
    with pytest.raises(gsa.GsError):
        p.run_pipeline("warp_total", 32, 0, 1, sub=99)


def test_divided_plan_file_round_trip(tmp_path):
    """§8f ranks 3 + 4: one binary plan file holds every sub-matrix's kernel"""
    r, c, v = random_coo(300, 90, 0.08, 7, empty=0.1)
    keep = (r < 100) | (r >= 160)
    r, c, v = r[keep], c[keep], v[keep]
    p = gsa.Plan.from_coo(300, 90, r, c, v)
    subs = p.divide_rows(60)
    pipes = ["merge_path", "tblock_warp_total", "thread_total", "balanced_warp_total"]
    for i, s in enumerate(subs):
        p.run_pipeline(pipes[i % len(pipes)], 8, 16, 1, sub=s)
    p.compile()
    f = tmp_path / "divided.gsplan"
    p.save(f)
    q = gsa.Plan.load(f)
    assert q.sub_matrices() == subs
    a, b = p.arrays(), q.arrays()
    assert sorted(a) == sorted(b)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    ia, ib = p.info(), q.info()
    for k in ("n_kernels", "rows", "cols", "nnz", "nnz_stored", "family", "kernel_name"):
        assert ia[k] == ib[k], k


# ---------------------------------------------------------------- row_nz_matrix_div_operator
def check_row_nz_division(M, K, r, c, v, init, mx):
    exp, err = ofi.run_pipeline(M, K, r, c, v, "row_nz_div", init, mx)
    p = gsa.Plan.from_coo(M, K, r, c, v)
    if err is not None:
        with pytest.raises(gsa.GsError):
            p.add_operator("row_nz_matrix_div_operator", init, mx, 2)
        return None
    p.add_operator("row_nz_matrix_div_operator", init, mx, 2)
    got = p.arrays()
    assert sorted(got) == sorted(exp)
    for k, a in exp.items():
        np.testing.assert_array_equal(got[k], a, err_msg=k)
    return p


def test_row_nz_division_hand_case():
    # row lengths 5,5,0,0,5,5 with windows from 4 (x2 up to 64): positions 0, 2, 4.
    # The entries move on one bucket at a time: row 4's first entry lands in bucket 1
    # (rows 2-3), its others in bucket 2 -- the reference's assignment loop
    # (div_row_indices_by_row_nnz.cc), restated as is
    r = np.repeat(np.array([0, 1, 4, 5], np.uint64), 5)
    c = np.tile(np.arange(5, dtype=np.uint64), 4)
    v = np.arange(1, 21, dtype=np.float32)
    p = check_row_nz_division(6, 5, r, c, v, 4, 64)
    a = p.arrays()
    assert [a[f"GLOBAL_META_begin_row_index_{s}"][0] for s in (1, 2, 3)] == [0, 2, 4]
    assert [a[f"GLOBAL_META_end_row_index_{s}"][0] for s in (1, 2, 3)] == [1, 3, 5]
    assert a["GLOBAL_META_nz_row_indices_1"].tolist() == [0] * 5 + [1] * 5
    assert a["GLOBAL_META_nz_row_indices_2"].tolist() == [4]
    assert a["GLOBAL_META_nz_row_indices_3"].tolist() == [4] * 4 + [5] * 5
    assert a["GLOBAL_META_nz_vals_2"].tolist() == [11.0]
    # rows stay in the parent's indexing: the sub-matrices compile as parent-indexed
    # (scratch outputs summed by the executor; GPU parity in test_gpu_row_nz.py)
    for s in p.sub_matrices():
        p.run_pipeline("warp_total", 32, 0, 1, sub=s)
    p.compile()
    # the sort-based pipelines fail like the reference's row-count assert
    # (reorder_val_by_index.cc:42: end_row_index - begin_row_index + 1 rows expected)
    q = check_row_nz_division(6, 5, r, c, v, 4, 64)
    with pytest.raises(gsa.GsError, match="row count"):
        q.run_pipeline("thread_total", 8, 4, 1, sub=3)


def test_row_nz_then_fixed_division_refused():
    # a fixed-interval division of a row_nz sub-matrix (rows in its parent's indexing) has
    # no row range to write to: compile refuses it
    r = np.repeat(np.array([0, 1, 4, 5], np.uint64), 5)
    c = np.tile(np.arange(5, dtype=np.uint64), 4)
    v = np.arange(1, 21, dtype=np.float32)
    p = gsa.Plan.from_coo(6, 5, r, c, v)
    p.add_operator("row_nz_matrix_div_operator", 4, 64, 2)
    try:
        subs = p.divide_rows(1, sub=3)
    except gsa.GsError:
        return  # the division itself may be invalid on such a sub-matrix
    for s in p.sub_matrices():
        p.run_pipeline("warp_total", 8, 0, 1, sub=s)
    with pytest.raises(gsa.GsError, match="not executable"):
        p.compile()
    assert subs


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("win", [(4, 64), (8, 32), (2, 1024), (16, 16)])
def test_row_nz_division_matches_oracle(seed, win):
    rng = np.random.default_rng(40 + seed)
    M, K = 120, 300
    # bands of similar row length (few positions) with some noise rows
    lens = np.repeat(rng.choice([0, 3, 12, 40, 90], size=6), 20)
    lens[rng.random(M) < 0.03 * seed] = 1
    rows = np.repeat(np.arange(M, dtype=np.uint64), lens)
    cols = np.concatenate([np.sort(rng.choice(K, size=n, replace=False)) for n in lens]).astype(np.uint64)
    if len(rows) == 0:
        return
    vals = rng.uniform(-1, 1, len(rows)).astype(np.float32)
    check_row_nz_division(M, K, rows, cols, vals, *win)
