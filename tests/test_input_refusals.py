"""CPU checks of the input edges at the boundary: what the reference's reader refuses
(no entries, struct.cc:258; unsorted rows, struct.cc:120-131) is refused here with an error
instead of an assert, and the malformed inputs the reference leaves undefined (a 0 or
non-numeric .mtx index, which its stoul turns into index -1; negative, non-integer or
mismatched COO arrays; indices past the device layouts' 32 bits) are refused before any plan
array is built.  Dims grow to the largest index + 1, as the reference derives them from the
entries (struct.cc:104-131)."""
import numpy as np
import pytest

import generalsparse_amd as gsa

HDR = "%%MatrixMarket matrix coordinate real general\n"
F32 = np.float32


def _mtx(tmp_path, body):
    p = tmp_path / "m.mtx"
    p.write_text(HDR + body)
    return str(p)


def test_empty_matrix_is_refused(tmp_path):
    e = np.zeros(0, np.int64)
    with pytest.raises(gsa.GsError, match="empty matrix"):
        gsa.Plan.from_coo(16, 16, e, e, np.zeros(0, F32))
    with pytest.raises(gsa.GsError, match="empty matrix"):
        gsa.Plan.from_mtx(_mtx(tmp_path, "5 5 0\n"))


@pytest.mark.parametrize("body", ["3 3 2\n0 1 1.0\n3 2 4.0\n",   # 0 in a 1-based file
                                  "3 3 1\n1 0 2.0\n",
                                  "3 3 2\n1 1 1.0\n3 x 4.0\n",   # non-numeric
                                  "3 3 1\n1 -2 1.0\n",
                                  "3 3 1\n1 4294967297 1.0\n",  # past 2^32
                                  "3 3 1\n1 4294967296 1.0\n"])  # index 2^32 - 1: a dim of 2^32
def test_malformed_mtx_indices_are_refused(tmp_path, body):
    with pytest.raises(gsa.GsError, match="mtx index"):
        gsa.Plan.from_mtx(_mtx(tmp_path, body))


def test_unsorted_rows_are_refused(tmp_path):
    with pytest.raises(gsa.GsError, match="row-sorted"):
        gsa.Plan.from_mtx(_mtx(tmp_path, "3 3 2\n3 1 1.0\n1 2 4.0\n"))
    with pytest.raises(gsa.GsError, match="row-sorted"):
        gsa.Plan.from_coo(3, 3, np.array([2, 0]), np.array([0, 1]), np.ones(2, F32))


@pytest.mark.parametrize("row,col,val,msg", [
    (np.array([-1]), np.array([0]), np.ones(1, F32), "negative row"),
    (np.array([0]), np.array([-3]), np.ones(1, F32), "negative col"),
    (np.array([0, 1]), np.array([0]), np.ones(2, F32), "lengths differ"),
    (np.array([0, 1]), np.array([0, 1]), np.ones(3, F32), "lengths differ"),
    (np.array([0.5]), np.array([0]), np.ones(1, F32), "integer array"),
    (np.array([0]), np.array([2 ** 33]), np.ones(1, F32), "out of range"),
    (np.array([0]), np.array([2 ** 32 - 1]), np.ones(1, F32), "out of range"),
])
def test_malformed_coo_is_refused(row, col, val, msg):
    with pytest.raises(gsa.GsError, match=msg):
        gsa.Plan.from_coo(4, 4, row, col, val)


def test_dims_grow_to_the_largest_index(tmp_path):
    p = gsa.Plan.from_coo(4, 4, np.array([0, 6]), np.array([9, 1]), np.ones(2, F32))
    assert (p.info()["rows"], p.info()["cols"]) == (7, 10)
    p = gsa.Plan.from_mtx(_mtx(tmp_path, "3 3 2\n1 1 1.0\n7 2 4.0\n"))
    assert (p.info()["rows"], p.info()["cols"]) == (7, 3)


def test_single_entry_and_spaced_lines(tmp_path):
    """a 1 x 1 matrix plans through the row pipelines; repeated spaces before an index are
    skipped (the reference's single-space split would read an empty token)"""
    p = gsa.Plan.from_coo(1, 1, np.array([0]), np.array([0]), np.array([2.0], F32))
    p.run_pipeline("block_total", 8, 40, 1)
    q = gsa.Plan.from_mtx(_mtx(tmp_path, "2 2 2\n1  1 1.0\n2 2 3.0\n"), ones_values=False)
    assert q.info()["nnz"] == 2


def test_experiments_keys_in_a_json_config_are_refused(tmp_path):
    """the release build refuses the experiments-build switches when they come
    from the JSON config file (GS_CONFIG / ./global_config.json) as it does in set_config, so a
    KS_POS8 plan can never reach the release build's grouped k_mfma_ks launch"""
    import os
    import subprocess
    import sys
    from build_flags import EXPERIMENTS
    if EXPERIMENTS:
        pytest.skip("the experiments build accepts these keys")
    cfg = tmp_path / "cfg.json"
    cfg.write_text('{"HALF": true, "KS_POS8": 1}\n')
    code = ("import generalsparse_amd as g\n"
            "try:\n    g.get_config('KS_NT')\nexcept g.GsError as e:\n    print('REFUSED', e)\n")
    env = dict(os.environ, GS_CONFIG=str(cfg))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert "REFUSED" in out.stdout and "KS_POS8" in out.stdout, out.stdout + out.stderr
    cfg.write_text('{"HALF": true, "KS_NT": 1}\n')
    code = "import generalsparse_amd as g\nprint('KS_NT', g.get_config('KS_NT'))\n"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert "KS_NT 1" in out.stdout, out.stdout + out.stderr
