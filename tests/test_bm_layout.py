"""k_mfma_bm's bitmap layout (host/device_layout.cc build_bm_tiles), decoded on the CPU from
the binary sidecars generate_final_program writes: every stored value lands at its
(row, column), nothing else is stored, the records' lane offsets and the step bases are
consistent.  The layout is this build's (no reference counterpart); the matrix it encodes
is the plan's canonical COO (fp16 values, duplicates summed)."""
import os
import re

import numpy as np
import pytest

import generalsparse_amd as gsa
from generalsparse_amd import datasets as ds
from build_flags import experiments

pytestmark = experiments


def _decode(d, M, K, tbr):
    rec = np.fromfile(os.path.join(d, "TBLOCK_META_mfma_bm_records_0.bin"), np.uint32).reshape(-1, 2)
    sb = np.fromfile(os.path.join(d, "TBLOCK_META_mfma_bm_step_base_0.bin"), np.uint32)
    val = np.fromfile(os.path.join(d, "TBLOCK_META_mfma_bm_values_0.bin"), np.uint16).view(np.float16)
    src = open(os.path.join(d, "kernel_file.hip")).read()
    m = re.search(r"k_mfma_bm<(\d+), (\d+), (\d+), \d+>.*\(uint32_t\)K, N, (\d+)u, (\d+)u, (\d+)u, 0u, d_ws", src)
    if m:
        CT, RT, W, S, NS, nwg = map(int, m.groups())
    else:
        m = re.search(r"k_mfma_bm2<(\d+), (\d+)>.*\(uint32_t\)K, N, (\d+)u, (\d+)u, (\d+)u, 0u, d_ws", src)
        assert m, "no k_mfma_bm / k_mfma_bm2 launch in the emitted program"
        CT, RT, S, NS, nwg = map(int, m.groups())
        W = RT
    nb = len(tbr) - 1
    assert nwg == nb * S and len(sb) == nb * S * NS + 1 and len(rec) == nb * S * NS * 64
    KR = 32 * NS
    assert S * KR >= K > (S - 1) * KR
    dense = np.zeros((M, K), np.float64)
    cnt = np.zeros((M, K), np.int64)
    lane = np.arange(64)
    for u in range(nb * S):
        g, q = divmod(u, S)
        r0, R = int(tbr[g]), int(tbr[g + 1] - tbr[g])
        for s in range(NS):
            x = u * NS + s
            w0, w1 = rec[x * 64:(x + 1) * 64, 0], rec[x * 64:(x + 1) * 64, 1]
            off = (w1 >> 16).astype(np.int64)
            masks = [((w0 >> (8 * t)) & 255) if t < 4 else ((w1 >> (8 * (t - 4))) & 255) for t in range(RT)]
            cnt_l = sum(np.array([bin(int(v)).count("1") for v in mk]) for mk in masks)
            np.testing.assert_array_equal(off, np.concatenate([[0], np.cumsum(cnt_l)[:-1]]))
            assert sb[x + 1] - sb[x] == cnt_l.sum()
            p = int(sb[x]) + off
            for t in range(RT):
                for bit in range(8):
                    on = ((masks[t] >> bit) & 1).astype(bool)
                    rows = 16 * t + lane % 16
                    cols = q * KR + 32 * s + 8 * (lane // 16) + bit
                    assert np.all(rows[on] < R) and np.all(cols[on] < K)
                    dense[r0 + rows[on], cols[on]] += val[p[on]]
                    cnt[r0 + rows[on], cols[on]] += 1
                    p = p + on
    assert np.all(val[int(sb[-1]):] == 0)   # the pad
    return dense, cnt, (CT, RT, W, S, NS)


@pytest.mark.parametrize("v2", [0, 1])
@pytest.mark.parametrize("p0,split,waves", [(80, 0, 8), (40, 0, 4), (96, 3, 8), (20, 1, 8), (7, 2, 4)])
def test_bm_layout_decodes_to_the_matrix(tmp_path, p0, split, waves, v2):
    M, K, N = 300, 500, 32
    row, col, val = ds.pruned_weight(M, K, 0.7, 31)
    old = {k: gsa.get_config(k) for k in ("MFMA_BM", "BM_SPLIT", "BM_WAVES", "HALF", "BM_V2")}
    try:
        gsa.set_config("MFMA_BM", 1)
        gsa.set_config("BM_SPLIT", split)
        gsa.set_config("BM_WAVES", waves)
        gsa.set_config("HALF", 1)
        gsa.set_config("BM_V2", v2)
        p = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, p0, 1).compile()
        d = p.generate_program(tmp_path, repeat=10)
        tbr = p.array("TBLOCK_META_first_row_indices_0")
    finally:
        for k, v in old.items():
            gsa.set_config(k, v)
    dense, cnt, (CT, RT, W, S, NS) = _decode(d, M, K, tbr)
    assert RT == (max(np.diff(tbr.astype(np.int64))) + 15) // 16
    assert W == (RT if v2 else waves)
    if split:
        assert S == split
    ref = np.zeros((M, K), np.float64)
    np.add.at(ref, (row.astype(np.int64), col.astype(np.int64)), val.astype(np.float16).astype(np.float64))
    assert cnt.max() == 1
    np.testing.assert_array_equal(cnt, (np.zeros((M, K), np.int64) + 0) + np.isin(
        np.arange(M * K), row.astype(np.int64) * K + col.astype(np.int64)).reshape(M, K))
    np.testing.assert_array_equal(dense, ref)
