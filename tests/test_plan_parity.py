"""Plan parity (CPU): the C++ plan builder in libgeneralsparse.so must produce
bit-identical plan arrays to the oracle for every canned pipeline
(token_test.cc test_spmm_*), and the C ABI must export what
include/generalsparse.h declares.  No GPU needed."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

import oracle_ffi as ofi

import generalsparse_amd as gsa
from generalsparse_amd import _lib
from generalsparse_amd import datasets as ds

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "hand_plans.json")


def oracle_params(name, N, p0, p1):
    """maps a product pipeline call to the oracle's parameters"""
    cf = p1 if p1 > 0 else 1
    if name == "thread_total":
        return p0 if p0 > 0 else 4
    if name == "tblock_warp_total_relative":
        return p0
    if name == "warp_segment":
        return min(N, 32)
    if name == "thread_bit_map":
        return N // cf if N // cf < 32 else 32
    if name in ("warp_bit_map", "warp_bit_map_interleaved"):  # token_test.cc:1277-1279
        return max(128 // min(max(1, N // cf), 32), 32)
    if name in ("tblock_bit_map", "tblock_bit_map_interleaved"):  # token_test.cc:1546-1547
        return 256 // min(max(1, N // cf), 32)
    return p0


def product_plan(M, K, row, col, val, name, N, p0=0, p1=0):
    p = gsa.Plan.from_coo(M, K, row, col, val)
    p.run_pipeline(name, N, p0, p1)
    return p


def compare(M, K, row, col, val, name, N, p0=0, p1=0):
    exp, err = ofi.run_pipeline(M, K, row, col, val, name, oracle_params(name, N, p0, p1),
                                p1 if name in ("merge_path", "tblock_warp_total_relative", "tblock_thread_total",
                                               "tblock_warp_thread_total") else 0)
    if err is not None:
        with pytest.raises(gsa.GsError):
            product_plan(M, K, row, col, val, name, N, p0, p1)
        return None
    p = product_plan(M, K, row, col, val, name, N, p0, p1)
    got = p.arrays()
    for key, arr in exp.items():
        assert key in got, f"{name}: product lacks {key}"
        np.testing.assert_array_equal(got[key].astype(np.float64) if arr.dtype == np.float64 else got[key],
                                      arr, err_msg=f"{name}: {key}")
    return p


def random_coo(M, K, density, seed, empty=0.2, trailing_empty=False):
    rng = np.random.default_rng(seed)
    mask = rng.random((M, K)) < density
    mask[rng.random(M) < empty] = False
    if trailing_empty:
        mask[-3:] = False
    r, c = np.nonzero(mask)
    v = rng.uniform(-1, 1, size=len(r)).astype(np.float32)
    return r.astype(np.uint64), c.astype(np.uint64), v


PIPES = [("thread_total", 32, 4, 1), ("thread_total", 8, 8, 1), ("warp_total", 32, 0, 1),
         ("block_total", 8, 0, 1), ("thread_bit_map", 32, 4, 1), ("thread_bit_map", 8, 4, 2),
         ("warp_segment", 32, 4, 1), ("warp_segment", 8, 4, 1), ("tblock_warp_total", 32, 4, 1),
         ("tblock_warp_total", 32, 7, 1), ("balanced_warp_total", 32, 64, 1), ("warp_bit_map", 32, 4, 1),
         ("tblock_bit_map", 32, 4, 1), ("balanced_block_total", 32, 64, 1), ("balanced_block_total", 8, 7, 1),
         ("balanced_thread_total", 8, 16, 1), ("merge_path", 8, 16, 1), ("merge_path", 8, 7, 2),
         ("merge_path", 32, 5, 3), ("merge_path", 8, 1, 1), ("merge_path", 8, 1024, 1),
         ("tblock_warp_total_relative", 32, 20, 2), ("tblock_warp_total_relative", 32, 7, 3),
         ("tblock_thread_total", 32, 16, 1), ("tblock_thread_total", 32, 20, 3), ("tblock_thread_total", 8, 5, 7),
         ("tblock_warp_thread_total", 32, 16, 1), ("tblock_warp_thread_total", 32, 20, 3),
         ("tblock_warp_thread_total", 8, 33, 5)]

# col-direction pipelines need rows long enough for the 64-nnz padding rule
COL_PIPES = [("warp_bit_map", 32, 4, 1), ("warp_bit_map", 8, 4, 2), ("warp_bit_map", 1, 4, 1),
             ("warp_bit_map_interleaved", 32, 4, 1), ("tblock_bit_map_interleaved", 8, 4, 1),
             ("tblock_bit_map", 32, 4, 1), ("tblock_bit_map", 128, 4, 1), ("tblock_bit_map", 2, 4, 1)]


@pytest.mark.parametrize("pipe", COL_PIPES, ids=lambda p: f"{p[0]}-N{p[1]}-{p[3]}")
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_col_direction_plans_bit_exact(pipe, seed):
    name, N, p0, p1 = pipe
    M, K = 150 + 31 * seed, 400
    r, c, v = random_coo(M, K, 0.25 + 0.1 * seed, seed, empty=0.1, trailing_empty=(seed == 2))
    p = compare(M, K, r, c, v, name, N, p0, p1)
    assert p is not None
    p.compile()


@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-N{p[1]}-{p[2]}-{p[3]}")
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_plan_arrays_bit_exact(pipe, seed):
    name, N, p0, p1 = pipe
    M, K = 120 + 17 * seed, 90
    r, c, v = random_coo(M, K, 0.08, seed, trailing_empty=(seed == 1))
    compare(M, K, r, c, v, name, N, p0, p1)


@pytest.mark.parametrize("pipe", PIPES, ids=lambda p: f"{p[0]}-N{p[1]}")
def test_plan_edge_shapes(pipe):
    name, N, p0, p1 = pipe
    cases = [
        (1, 1, np.array([0], np.uint64), np.array([0], np.uint64)),            # single nnz
        (1, 70, np.zeros(70, np.uint64), np.arange(70, dtype=np.uint64)),     # one long row
        (70, 1, np.arange(70, dtype=np.uint64), np.zeros(70, np.uint64)),     # one column
        (5, 5, np.array([4], np.uint64), np.array([2], np.uint64)),            # leading empty rows
    ]
    for M, K, r, c in cases:
        v = np.linspace(-1, 1, len(r)).astype(np.float32)
        compare(M, K, r, c, v, name, N, p0, p1)


def test_hand_derived_fixtures_through_product():
    g = json.load(open(GOLDEN))
    back = {"thread_total": (32, 4, 1), "warp_total": (32, 0, 1), "block_total": (8, 0, 1),
            "merge_path": (8, 0, 1), "balanced_block_total": (32, 0, 1), "balanced_thread_total": (8, 0, 1),
            "warp_bit_map_interleaved": (32, 4, 1), "tblock_warp_total_relative": (32, 4, 2),
            "tblock_warp_total": (32, 4, 1), "balanced_warp_total": (32, 16, 1),
            "warp_bit_map": (32, 4, 1), "tblock_bit_map": (32, 4, 1), "tblock_bit_map_interleaved": (32, 4, 1),
            "tblock_col_thread_interleaved": (32, 4, 2), "warp_col_thread_interleaved": (32, 4, 2),
            "tblock_col_thread_maxpad": (32, 4, 2), "tblock_thread_total_maxpad": (32, 4, 1),
            "tblock_thread_total": (32, 4, 1), "tblock_warp_thread_total": (32, 4, 1)}
    for case in g["cases"]:
        m = g["matrices"][case["matrix"]]
        row = np.array([e[0] for e in m["entries"]], np.uint64)
        col = np.array([e[1] for e in m["entries"]], np.uint64)
        val = np.arange(1, len(row) + 1, dtype=np.float32)
        name = case["pipeline"]
        if name in ("warp_segment", "thread_bit_map"):
            N, p0, p1 = case["p0"], 4, 1  # VW = min(N, 32) = fixture VW
        elif name in ("tblock_balanced_thread_total", "tblock_thread_total_colpad", "nnz_tblock_bitmap",
                      "nnz_tblock_warp_bitmap"):
            N, p0, p1 = 32, case["p0"], case.get("p1", 0)  # the fixture's own parameters
        else:
            N, p0, p1 = back[name]
            if name in ("tblock_warp_total", "balanced_warp_total", "merge_path", "balanced_block_total",
                        "balanced_thread_total", "tblock_warp_total_relative", "tblock_thread_total",
                        "tblock_warp_thread_total", "tblock_col_thread_interleaved", "warp_col_thread_interleaved", "tblock_col_thread_maxpad",
                        "tblock_thread_total_maxpad"):
                p0 = case["p0"]
            if name in ("merge_path", "tblock_warp_total_relative", "tblock_thread_total", "tblock_warp_thread_total",
                        "tblock_col_thread_interleaved", "warp_col_thread_interleaved", "tblock_col_thread_maxpad",
                        "tblock_thread_total_maxpad"):
                p1 = case["p1"]
        if case.get("expect_error"):
            with pytest.raises(gsa.GsError):
                product_plan(m["M"], m["K"], row, col, val, name, N, p0, p1)
            continue
        got = product_plan(m["M"], m["K"], row, col, val, name, N, p0, p1).arrays()
        for key, exp in case["expect"].items():
            np.testing.assert_array_equal(got[key].astype(np.float64), np.asarray(exp, np.float64), err_msg=key)


def test_operator_surface_matches_pipeline():
    """The same plan through gs_plan_add_operator (reference class names and
    constructor arguments) as through the canned pipeline."""
    M, K = 60, 50
    r, c, v = random_coo(M, K, 0.1, 5)
    a = gsa.Plan.from_coo(M, K, r, c, v)
    gsa.set_config("DENSE_MATRIX_SIZE", 32)
    a.add_operator("sort_operator")
    a.add_operator("fixed_interval_row_direction_thread_blocking_operator", 1, 0, 0, 0, 0, 1, 4)
    a.add_operator("thread_total_reduce_operator", 0, 4, 1)
    b = product_plan(M, K, r, c, v, "thread_total", 32, 4, 1)
    ga, gb = a.arrays(), b.arrays()
    assert set(ga) == set(gb)
    for k in ga:
        np.testing.assert_array_equal(ga[k], gb[k], err_msg=k)
    assert "sort_operator" in a.log()


def test_operator_validity_rules():
    """name-substring validity (thread_total_reduce_operator.cc:14-40 etc.)"""
    M, K = 30, 30
    r, c, v = random_coo(M, K, 0.2, 9)
    p = gsa.Plan.from_coo(M, K, r, c, v)
    with pytest.raises(gsa.GsError):  # no thread-level distributing op yet
        p.add_operator("thread_total_reduce_operator", 0, 4, 1)
    p.add_operator("fixed_interval_nnz_direction_thread_blocking_operator", 32, 0, 0, 1)
    with pytest.raises(gsa.GsError):  # "nnz" distributing op forbids thread_total
        p.add_operator("thread_total_reduce_operator", 0, 4, 1)
    with pytest.raises(gsa.GsError):  # sort after distributing is invalid (sort_operator.cc:20-45)
        p.add_operator("sort_operator")
    with pytest.raises(gsa.GsError):  # warp_segment needs thread_bit_map first
        p.add_operator("warp_segment_reduce_operator", 1, 0, 0)
    p.add_operator("thread_bit_map_operator", 1, 8, 4, 1)
    p.add_operator("warp_segment_reduce_operator", 1, 0, 0)
    p.compile()
    assert p.info()["kernel_name"].startswith("k_bitmap_segment")


def test_interlance_storage_validity():
    """interlance_storage_operator.cc:56-141: only after a col-direction thread blocking
    padded to its size, once, before any implementing operator"""
    M, K = 20, 300
    r, c, v = random_coo(M, K, 0.5, 3, empty=0.0)
    gsa.set_config("DENSE_MATRIX_SIZE", 32)
    p = gsa.Plan.from_coo(M, K, r, c, v)
    p.add_operator("fixed_interval_col_direction_thread_blocking_operator", 64, 0, 0, 0, 0)  # no padding
    with pytest.raises(gsa.GsError):
        p.add_operator("interlance_storage_operator")
    q = gsa.Plan.from_coo(M, K, r, c, v)
    q.add_operator("fixed_interval_col_direction_thread_blocking_operator", 64, 0, 0, 1, 0)
    q.add_operator("interlance_storage_operator")
    with pytest.raises(gsa.GsError):
        q.add_operator("interlance_storage_operator")
    q.add_operator("thread_total_reduce_operator", 1, 4, 1)
    q.add_operator("warp_bit_map_operator", 1, 1, 1)
    q.compile()
    assert q.info()["kernel_name"].endswith("+interleaved")
    a = q.arrays()
    n, sz = len(a["GLOBAL_META_nz_col_indices_0"]), int(a["GLOBAL_META_BMT_size_of_each_blk_0"][0])
    nb = n // sz
    perm = np.array([b + i * nb for b in range(nb) for i in range(sz)])
    np.testing.assert_array_equal(a["GLOBAL_META_nz_col_indices_after_interlance_storage_0"][perm],
                                  a["GLOBAL_META_nz_col_indices_0"])


def test_mtx_reader_parity(tmp_path):
    M, K = 40, 33
    r, c, v = random_coo(M, K, 0.15, 11, trailing_empty=True)
    path = tmp_path / "m.mtx"
    ds.write_mtx(path, M, K, r, c, v)
    L = ofi.lib()

    class Coo(ctypes.Structure):
        _fields_ = [("nnz", ctypes.c_uint64), ("row", ctypes.POINTER(ctypes.c_uint64)),
                    ("col", ctypes.POINTER(ctypes.c_uint64)), ("val", ctypes.POINTER(ctypes.c_float)),
                    ("max_row_index", ctypes.c_uint64), ("max_col_index", ctypes.c_uint64)]
    for ones in (1, 0):
        co = Coo()
        assert L.or_read_mtx(str(path).encode(), ones, ctypes.byref(co)) == 0
        p = gsa.Plan.from_mtx(path, ones_values=bool(ones))
        rows = np.ctypeslib.as_array(co.row, (co.nnz,)).copy()
        vals = np.ctypeslib.as_array(co.val, (co.nnz,)).copy()
        np.testing.assert_array_equal(p.array("GLOBAL_META_nz_row_indices_0"), rows)
        np.testing.assert_array_equal(p.array("GLOBAL_META_nz_vals_0"), vals.astype(np.float64))
        assert p.array("GLOBAL_META_origin_row_num_-1")[0] == M
        L.or_coo_free(ctypes.byref(co))


def test_unsorted_mtx_rejected(tmp_path):
    path = tmp_path / "bad.mtx"
    path.write_text("3 3 2\n2 1 1.0\n1 1 1.0\n")
    with pytest.raises(gsa.GsError):
        gsa.Plan.from_mtx(path)


def test_c_abi_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "generalsparse.h")).read()
    declared = set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", hdr))
    L = _lib.load()
    for sym in sorted(declared):
        assert hasattr(L, sym), sym
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_generate_program(tmp_path):
    M, K = 50, 40
    r, c, v = random_coo(M, K, 0.1, 3)
    p = product_plan(M, K, r, c, v, "thread_total", 32, 4, 1)
    p.compile()
    d = p.generate_program(tmp_path, repeat=10)
    files = set(os.listdir(d))
    assert {"kernel_file.hip", "make_kernel.sh", "kernel_lib.hpp", "THREAD_META_first_nz_indices_0",
            "GLOBAL_META_original_nz_row_indices_0"} <= files
    fn = np.loadtxt(os.path.join(d, "THREAD_META_first_nz_indices_0"), dtype=np.uint64)
    np.testing.assert_array_equal(fn, p.array("THREAD_META_first_nz_indices_0"))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
def test_generate_program_row_chunks_compiles(tmp_path):
    """the emitted standalone program of a col-direction plan (K5) is valid HIP"""
    M, K = 40, 300
    r, c, v = random_coo(M, K, 0.4, 4)
    p = product_plan(M, K, r, c, v, "warp_bit_map", 32, 4, 1)
    p.compile()
    d = p.generate_program(tmp_path, repeat=10)
    src = open(os.path.join(d, "kernel_file.hip")).read()
    assert "k_row_chunks" in src and "k_finalize_rows" in src
    assert "WARP_META_bit_map_of_thread_0" in os.listdir(d)
    import subprocess
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-c",
                           "kernel_file.hip", "-o", "kernel_file.o"], cwd=d)


@pytest.mark.parametrize("name,p0,p1", [("merge_path", 64, 1), ("balanced_thread_total", 16, 1)])
def test_generate_program_new_families_compile(tmp_path, name, p0, p1):
    """the emitted programs of a merge-path plan (k_merge_path + k_merge_fixup) and of
    multi-row balanced BMTs (wave per row group) are valid HIP"""
    M, K = 60, 300
    r, c, v = random_coo(M, K, 0.3, 6, trailing_empty=False)
    p = product_plan(M, K, r, c, v, name, 8, p0, p1)
    p.compile()
    d = p.generate_program(tmp_path, repeat=10)
    src = open(os.path.join(d, "kernel_file.hip")).read()
    assert ("k_merge_path" in src and "k_merge_fixup" in src) if name == "merge_path" else "k_warp_rows" in src
    import subprocess
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-c",
                           "kernel_file.hip", "-o", "kernel_file.o"], cwd=d)


def test_synthetic_generators_shapes():
    r, c, v = ds.pruned_weight(64, 48, 0.7, 13)
    assert len(r) == round(0.3 * 64 * 48) and np.all(np.diff(r.astype(np.int64)) >= 0)
    r, c, v = ds.two_four(8, 16, 30)
    assert len(r) == 8 * 8
    assert np.all(np.bincount((c // 4 + 4 * r).astype(np.int64)) == 2)
    r, c, v = ds.rmat(1024, 5000, 1)
    assert len(r) <= 5000 and np.all(np.diff(r.astype(np.int64)) >= 0)


@pytest.mark.parametrize("name,N,p0,p1", [("tblock_warp_total", 32, 20, 2), ("merge_path", 8, 64, 1),
                                          ("warp_bit_map_interleaved", 32, 4, 1), ("warp_segment", 32, 4, 1)])
def test_binary_plan_file_round_trip(tmp_path, name, N, p0, p1):
    """§8f rank 4: a compiled plan saved to one binary file loads back with every plan
    array bit-identical and the same kernel selection"""
    M, K = 150, 400
    r, c, v = random_coo(M, K, 0.2, 8, empty=0.1)
    p = product_plan(M, K, r, c, v, name, N, p0, p1)
    p.compile()
    f = tmp_path / "plan.gsplan"
    p.save(f)
    q = gsa.Plan.load(f)
    assert q.info()["kernel_name"] == p.info()["kernel_name"]
    a, b = p.arrays(), q.arrays()
    assert set(a) == set(b)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    bad = tmp_path / "bad.gsplan"
    bad.write_bytes(b"not a plan")
    with pytest.raises(gsa.GsError):
        gsa.Plan.load(bad)


@pytest.mark.parametrize("nt", [0, 1])
def test_generate_program_carries_nontemporal_variants(tmp_path, nt):
    """KS_NT / NM_NT reach the emitted program: it launches the same k_mfma_ks / k_nm_mfma
    instantiation gs_spmm does (the 9th / 4th template argument; k_nm_mfma's 5th: tiles per workgroup)"""
    old = {k: gsa.get_config(k) for k in ("HALF", "KS_NT", "NM_NT")}
    try:
        gsa.set_config("HALF", 1)
        gsa.set_config("KS_NT", nt)
        gsa.set_config("NM_NT", nt)
        (tmp_path / "ks").mkdir()
        (tmp_path / "nm").mkdir()
        r, c, v = ds.pruned_weight(320, 1024, 0.7, 41)
        p = gsa.Plan.from_coo(320, 1024, r, c, v).run_pipeline("block_total", 32, 40, 1).compile()
        src = open(os.path.join(p.generate_program(tmp_path / "ks", repeat=10), "kernel_file.hip")).read()
        assert re.search(r"gsk::k_mfma_ks<2, 3, 8, \d, \d, false, true, false%s>" % (", 1" if nt else ""), src), src[:2000]
        r, c, v = ds.two_four(256, 512, 41)
        p = gsa.Plan.from_coo(256, 512, r, c, v).run_pipeline("col_direction_nm", 32, 32, 1).compile()
        src = open(os.path.join(p.generate_program(tmp_path / "nm", repeat=10), "kernel_file.hip")).read()
        # 16 tiles: 8 workgroups of 2 tiles (the upload's nm_tiles_for rule, TT = last argument)
        assert ("gsk::k_nm_mfma<2, 0, 32, %s, 2>" % ("true" if nt else "false")) in src, src[:2000]
    finally:
        for k, val in old.items():
            gsa.set_config(k, val)
