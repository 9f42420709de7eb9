"""§8f rank 1: the reference's model-driven index compression (code_generator.cc:
2618-3063).  The product's decision and parameters equal the oracle's restatement on
hand-made arrays (one per compressor, with the values worked out by hand from the cited
rules) and on every integer array of real plans; exact formulas decode back to the array;
the reference's acceptance quirks are kept (and flagged not exact)."""
import numpy as np
import pytest

import oracle_ffi as ofi

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds

U8, U16, U32, U64 = 1, 6, 11, 16  # gs data_type codes (struct.hpp order)

HAND = [
    # (array, storage type, expected kind, expected params subset)
    ([0, 20, 40, 60, 80], U64, "linear", {"coef": 20, "intercept": 0}),
    ([7, 7, 7, 7], U64, "linear", {"coef": 0, "intercept": 7}),
    ([3, 3, 9, 9, 9, 4], U64, "branch", {}),                        # 3 runs < 5
    # the cycle is the LAST index holding a[0] (:2684-2691): two periods pass, three do not
    ([5, 6, 7, 5, 6, 7], U64, "cycle_linear", {"coef": 1, "intercept": 5, "cycle": 3}),
    # 5 runs: branch (tried before) rejects it
    ([0, 0, 2, 2, 4, 4, 6, 6, 8, 8], U64, "cycle_increase", {"cycle": 2, "coef": 2, "intercept": 0}),
    ([100, 201, 299, 402, 500, 603, 699, 800, 901, 999], U64, "residual", {}),
    ([1, 9, 2, 8, 3, 7], U8, "none", {}),                          # 6 runs, no model, u8 already
]


@pytest.mark.parametrize("case", range(len(HAND)))
def test_hand_arrays_oracle_and_product_agree(case):
    a, t, kind, want = HAND[case]
    ok, op, ores = ofi.index_compression(a, t)
    pk, pp, exact = gsa.index_compression_of_array(a, t)
    assert ok == pk == kind
    for k, v in want.items():
        assert op[k] == pp[k] == v, (k, op, pp)
    if kind == "residual":
        assert op["aa"] == pp["aa"] and op["bb"] == pp["bb"]
        dec = [(pp["aa"] * i + pp["bb"] + int(ores[i])) & ((1 << 64) - 1) for i in range(len(a))]
        assert dec == a and exact
    if kind in ("linear", "cycle_linear", "cycle_increase"):
        assert exact


def test_reference_quirk_cycle_increase_is_not_exact():
    """if_cycle_increase_compress only checks divisibility (:2748-2757): this array is
    accepted although (i/2)*2 gives 4 at i=4; the build flags it and keeps the array"""
    a = [0, 0, 2, 2, 6, 6, 12, 12, 24, 24]
    assert ofi.index_compression(a)[0] == "cycle_increase"
    kind, p, exact = gsa.index_compression_of_array(a)
    assert kind == "cycle_increase" and not exact


def test_reference_quirk_cycle_linear_three_periods():
    """with three periods the last a[0] sits at 6, (a[3]-a[0])/3 = 0 != coef: rejected (:2700-2711)"""
    a = [5, 6, 7, 5, 6, 7, 5, 6, 7]
    assert ofi.index_compression(a)[0] == gsa.index_compression_of_array(a)[0] != "cycle_linear"


def test_random_arrays_agree():
    rng = np.random.default_rng(3)
    for trial in range(200):
        n = int(rng.integers(2, 40))
        shape = trial % 5
        if shape == 0:
            a = rng.integers(0, 1000, n)
        elif shape == 1:
            a = np.repeat(rng.integers(0, 50, 3), n // 3 + 1)[:n]
        elif shape == 2:
            a = (np.arange(n) % int(rng.integers(1, 6))) * int(rng.integers(1, 4)) + int(rng.integers(0, 9))
        elif shape == 3:
            a = (np.arange(n) // int(rng.integers(1, 4))) * int(rng.integers(1, 5))
        else:
            a = np.arange(n) * 37 + rng.integers(0, 5, n)
        a = a.astype(np.uint64)
        for t in (U8, U16, U32, U64):
            ok, op, ores = ofi.index_compression(a, t)
            pk, pp, exact = gsa.index_compression_of_array(a, t)
            assert ok == pk, (a, t, ok, pk)
            if ok in ("linear", "cycle_linear", "cycle_increase"):
                assert (op["coef"], op["intercept"], op["cycle"]) == (pp["coef"], pp["intercept"], pp["cycle"])
            if ok == "residual":
                assert (op["aa"], op["bb"]) == (pp["aa"], pp["bb"])


def test_plan_arrays_compress_when_enabled():
    """MODEL_DRIVEN_COMPRESS on: every integer array of a row-blocked plan gets the
    oracle's decision; the BMTB starts of fixed blocking are linear; a residual adds
    <key>_res to the plan; off (the reference's default: the key is missing) -> none"""
    M, K = 400, 300
    r, c, v = ds.random_rows(M, K, 8.0, seed=4)
    gsa.set_config("MODEL_DRIVEN_COMPRESS", 1)
    try:
        p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("tblock_warp_total", 32, 20, 2)
        kind, expr, exact = p.index_compression("TBLOCK_META_first_row_indices_0")
        assert kind == "linear" and exact and expr == "20 * (i)"
        for key, arr in p.arrays().items():
            if arr.dtype != np.uint64 or len(arr) < 2 or key.endswith("_res_0"):
                continue
            k, e, ex = p.index_compression(key)
            ok, op, ores = ofi.index_compression(arr, 16 if arr.max() > 4294967295 else
                                                 (11 if arr.max() > 65535 else (6 if arr.max() > 255 else 1)))
            assert k == ok, (key, k, ok)
            if k == "residual":
                np.testing.assert_array_equal(p.array(key[:-2] + "_res_0"), ores)
    finally:
        gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)
    q = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("tblock_warp_total", 32, 20, 2)
    assert q.index_compression("TBLOCK_META_first_row_indices_0")[0] == "none"


def test_emitted_program_uses_exact_formulas(tmp_path):
    """with MODEL_DRIVEN_COMPRESS the generated program computes the compressible plan
    arrays (here the BMTB / BMW row starts of fixed blocking) and still compiles"""
    import os
    import subprocess
    M, K = 100, 300
    r, c, v = ds.random_rows(M, K, 6.0, seed=2)
    gsa.set_config("MODEL_DRIVEN_COMPRESS", 1)
    try:
        p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("tblock_warp_total", 32, 20, 2).compile()
        d = p.generate_program(tmp_path, repeat=10)
    finally:
        gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)
    src = open(os.path.join(d, "kernel_file.hip")).read()
    assert '"TBLOCK_META_first_row_indices_0"' in src and "20 * (i)" in src
    # the kernel evaluates the BMW row starts and the BMTB -> BMW map (5 BMTBs of 10 BMWs):
    # both linear, passed as gsk::idx_formula arguments, their arrays never uploaded
    assert "const gsk::idx_formula F1 = gsk::idx_formula{1u, 10u, 0u, 1u," in src
    assert "const gsk::idx_formula F0 = gsk::idx_formula{1u," in src
    assert "F0.kind ? nullptr : up(u32(wr))" in src and "(d_a0, F0, d_a1, F1, d_a2," in src
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-c",
                           "kernel_file.hip", "-o", "kernel_file.o"], cwd=d)
