"""CPU check of the k_mfma_ks upload layout through the emitted program's binary sidecars
(device_layout.cc build_ks_tiles): the step records and entry groups decode back to the
plan's matrix exactly, and with KS_HEAD the head steps (each wave's first kKsDepth k-steps)
sit at their fixed, padded slots -- record = ((g * S + q) * min(W * D, NS) + s) * GH -- with only
zero-row padding after their entries.  The emitted launch carries GH in prio bits 8..17."""
import os
import re

import numpy as np
import pytest

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds

RS = 48  # halfwords per wave-image row (kKsStride / 2)


def _emit(tmp_path, M, K, r, c, v, rows, head, split=0):
    keys = ("HALF", "KS_HEAD", "KS_SPLIT")
    old = {k: gsa.get_config(k) for k in keys}
    try:
        gsa.set_config("HALF", 1)
        gsa.set_config("KS_HEAD", head)
        gsa.set_config("KS_SPLIT", split)
        p = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("block_total", 32, rows, 1).compile()
        d = p.generate_program(tmp_path, repeat=10)
        tbr = p.array("TBLOCK_META_first_row_indices_0").astype(np.int64)
    finally:
        for k, val in old.items():
            gsa.set_config(k, val)
    return d, tbr


def _decode(d, M, K, tbr):
    src = open(os.path.join(d, "kernel_file.hip")).read()
    m = re.search(r"gsk::k_mfma_ks<(\d+), (\d+), (\d+), (\d+), (\d+)", src)
    CT, RT, W, D, MAXG = map(int, m.groups())
    m = re.search(r"\(uint32_t\)K, N, (\d+)u, (\d+)u, (\d+)u, 0u, d_ws, d_arr, nullptr, (\d+)u\)", src)
    S, NS, nwg, prio = map(int, m.groups())
    GH = (prio >> 8) & 0x3FF
    rd = lambda n, t: np.fromfile(os.path.join(d, n), dtype=t)
    steps = rd("TBLOCK_META_mfma_ks_steps_0.bin", np.uint32).reshape(-1, 2)
    pos = rd("TBLOCK_META_mfma_ks_entry_pos_0.bin", np.uint16).reshape(-1, 8)
    val = rd("TBLOCK_META_mfma_ks_entry_val_0.bin", np.uint16).reshape(-1, 8).view(np.float16)
    nb = len(tbr) - 1
    assert nwg == nb * S and len(steps) == nb * S * NS
    dense = np.zeros((M, K), np.float64)
    HS = min(W * D, NS)
    for g in range(nb):
        for q in range(S):
            u = g * S + q
            for s in range(NS):
                first, cnt = (int(x) for x in steps[u * NS + s])
                if GH and s < HS:
                    assert first == (u * HS + s) * GH and cnt <= GH, (u, s, first, cnt, GH)
                    pad = pos[first + cnt:first + GH]
                    assert np.all(pad // RS == 16 * RT) and np.all(val[first + cnt:first + GH] == 0)
                pp = pos[first:first + cnt].reshape(-1).astype(np.int64)
                vv = val[first:first + cnt].reshape(-1).astype(np.float64)
                row, colw = pp // RS, pp % RS
                live = row < 16 * RT
                assert np.all(vv[~live] == 0)
                assert np.all(row[live] < tbr[g + 1] - tbr[g]) and np.all(colw[live] < 32)
                np.add.at(dense, (tbr[g] + row[live], q * NS * 32 + 32 * s + colw[live]), vv[live])
    return dense, GH, (S, NS, W, D)


@pytest.mark.parametrize("rows,split", [(40, 0), (40, 1), (112, 0), (80, 3)])
@pytest.mark.parametrize("head", [0, 1])
def test_ks_layout_decodes_to_the_matrix(tmp_path, rows, split, head):
    M, K = 640, 4096
    r, c, v = ds.pruned_weight(M, K, 0.7, 51)
    d, tbr = _emit(tmp_path, M, K, r, c, v, rows, head, split)
    dense, GH, _ = _decode(d, M, K, tbr)
    ref = np.zeros((M, K), np.float64)
    np.add.at(ref, (r.astype(np.int64), c.astype(np.int64)), v.astype(np.float16).astype(np.float64))
    np.testing.assert_array_equal(dense, ref)
    if not head:
        assert GH == 0
    elif split == 1:  # 128 k-steps per unit: the 16 head slots cost a few % of padding
        assert GH > 0, GH


def test_ks_head_refused_when_padding_is_costly(tmp_path):
    """a plan whose head steps hold far more groups than the rest (the first 32 columns dense)
    keeps every step on its record: GH = 0"""
    M, K = 640, 4096
    r, c, v = ds.pruned_weight(M, K, 0.8, 52)
    dense_r, dense_c = np.meshgrid(np.arange(M), np.arange(32), indexing="ij")
    key = np.unique(np.concatenate([r.astype(np.int64) * K + c, dense_r.ravel() * K + dense_c.ravel()]))
    r2, c2 = (key // K).astype(np.int64), (key % K).astype(np.int64)
    v2 = np.random.default_rng(4).standard_normal(len(key)).astype(np.float32)
    d, tbr = _emit(tmp_path, M, K, r2, c2, v2, 40, 1, split=1)
    _, GH, (S, NS, W, D) = _decode(d, M, K, tbr)
    assert S == 1 and GH == 0


def test_ks_head_on_the_c2_plan(tmp_path):
    """the driver's C2 plan (block_total(40,1), 2 K ranges of 80 k-steps) takes the head layout"""
    M = K = 5120
    r, c, v = ds.pruned_weight(M, K, 0.7, 13)
    d, tbr = _emit(tmp_path, M, K, r, c, v, 40, 1)
    dense, GH, (S, NS, W, D) = _decode(d, M, K, tbr)
    assert (S, NS, W, D) == (2, 80, 8, 2) and GH > 0
    ref = np.zeros((M, K), np.float64)
    np.add.at(ref, (r.astype(np.int64), c.astype(np.int64)), v.astype(np.float16).astype(np.float64))
    np.testing.assert_array_equal(dense, ref)
