"""Bit-exact known answers at full size for the plans the measured lines run.

The reference's own known answer (all-ones A and B => C[i][j] = nnz(row i), code_generator.cc:633-637,
checked exactly by cuda_code/kernel_lib.hpp:884-921) is generalised here to small integers:
A's values in {-2, -1, 1, 2} on the measured sparsity pattern, B in {-2, ..., 2}.  Every product
and every partial sum is an integer below 2^24, so any fp32-accumulating kernel -- whatever its
summation order, K ranges or slab combine -- computes the exact integer and rounds it to fp16
once: C must equal fp16(exact) bit for bit.  Unlike the all-ones case, a nonzero landing in the
wrong column or row, a dropped or a doubled nonzero all change the answer.  The exact product is
a float64 dense matmul on the GPU (integers below 2^53: exact).

Cases:
- C2 as the driver's line runs it: block_total(40,1) on k_mfma_ks with KS_NT=1, two K ranges,
  head steps on (asserted in plan.info()), plus the all-ones known answer on the same plan;
- the north_star layer as bench.py runs it: OPT-30B 70% (4 x attn, fc1, fc2) on block_total(112,1),
  one k_mfma_ks_group launch of six entries;
- C3: OPT-30B fc1 2:4 on k_nm_mfma at N = 128 and N = 8.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import batch as bt  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def int_values(n, seed):
    """A's values: integers in {-2, -1, 1, 2} (exact in fp16)"""
    return np.random.default_rng(seed).choice(np.array([-2.0, -1.0, 1.0, 2.0], np.float32), n)


def int_B(K, N, seed):
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    return torch.randint(-2, 3, (K, N), device=DEV, generator=g).half()


def exact_fp16(M, K, row, col, val, B):
    """fp16(A @ B) from the exact integer product (float64 dense matmul on the GPU)"""
    A = torch.zeros((M, K), dtype=torch.float64, device=DEV)
    A[torch.from_numpy(row.astype(np.int64)).to(DEV), torch.from_numpy(col.astype(np.int64)).to(DEV)] = \
        torch.from_numpy(val.astype(np.float64)).to(DEV)
    out = A @ B.double()
    del A
    assert out.abs().max().item() < 65504  # representable: the fp16 rounding is the only one
    ref = out.half()
    del out
    torch.cuda.empty_cache()
    return ref


def build(M, K, row, col, val, pipeline, p0, p1, N, over=None):
    over = over or {}
    old = {k: gsa.get_config(k) for k in over}
    try:
        for k, v in over.items():
            gsa.set_config(k, v)
        return gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipeline, N, p0, p1).compile().upload("f16", 0)
    finally:
        for k, v in old.items():
            gsa.set_config(k, v)


def assert_bit_exact(C, ref, what):
    bad = (C.view(torch.int16) != ref.view(torch.int16))
    n_bad = int(bad.sum().item())
    if n_bad:
        i = bad.nonzero()[0].tolist()
        raise AssertionError(f"{what}: {n_bad} elements differ, first at {i}: {C[i[0], i[1]].item()} vs "
                             f"{ref[i[0], i[1]].item()}")


def test_c2_driver_plan_integer_known_answer():
    """C2 (OPT-13B q_proj stand-in 5120^2, 70%) on the driver's plan: block_total(40,1),
    KS_NT=1, 2 K ranges, head steps -- integer known answer and the all-ones known answer,
    both bit for bit, and a relaunch into a NaN-filled C"""
    M = K = 5120
    N = 32
    row, col, _ = ds.pruned_weight(M, K, 0.7, 13)
    val = int_values(len(row), 5)
    plan = build(M, K, row, col, val, "block_total", 40, 1, N, {"KS_NT": 1})
    info = plan.info()
    assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == 2, info
    assert info["ks_nt"] == 1 and info["ks_head_groups"] > 0, info
    B = int_B(K, N, 3)
    ref = exact_fp16(M, K, row, col, val, B)
    C = plan.spmm(B)
    torch.cuda.synchronize()
    assert_bit_exact(C, ref, "C2 integer")
    C2 = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float16)
    plan.spmm(B, C=C2)
    torch.cuda.synchronize()
    assert_bit_exact(C2, ref, "C2 integer relaunch")
    plan.device_status()
    plan.free()
    # the reference's own known answer on the same plan shape (values := 1, B := 1)
    ones = np.ones(len(row), np.float32)
    plan = build(M, K, row, col, ones, "block_total", 40, 1, N, {"KS_NT": 1})
    assert plan.info()["ksplit"] == 2 and plan.info()["ks_head_groups"] > 0
    C = plan.spmm(torch.ones((K, N), device=DEV, dtype=torch.float16))
    torch.cuda.synchronize()
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    want = torch.from_numpy(np.repeat(nnz_row[:, None], N, axis=1)).half().to(DEV)
    assert_bit_exact(C, want, "C2 all-ones")
    plan.free()


def test_headline_layer_grouped_integer_known_answer():
    """The north_star layer (OPT-30B 70%) as bench.py's north_star object runs it: every shape
    on block_total(112,1) (bench.HEADLINE_CHOICE), one gsa.Batch = ONE k_mfma_ks_group launch of
    six entries; every C equals fp16 of the exact integer product"""
    N = 32
    plans, entries, refs = {}, [], []
    for k in ("attn", "fc1", "fc2"):
        m, n = bt.C5_SHAPES[k]
        row, col, _ = ds.pruned_weight(m, n, 0.7, bt.shape_seed(0, k))
        val = int_values(len(row), 17 + len(plans))
        p = build(m, n, row, col, val, "block_total", 112, 1, N)
        info = p.info()
        assert info["device_kernel"] == "k_mfma_ks" and info["ksplit"] == (1 if k == "fc1" else 4), info
        if k == "attn":
            for _ in range(3):
                p.add_replica()
        plans[k] = (p, row, col, val)
    for slot, k in enumerate(bt.C5_SLOTS):
        p, row, col, val = plans[k]
        m, n = bt.C5_SHAPES[k]
        B = int_B(n, N, 100 + slot)
        C = torch.full((m, N), float("nan"), device=DEV, dtype=torch.float16)
        entries.append((p, bt.C5_SLOTS[:slot].count(k), B, C))
        refs.append(exact_fp16(m, n, row, col, val, B))
    bat = gsa.Batch(entries, N)
    assert bat.launches() == [6], bat.launches()
    bat.run(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for slot, ((p, rep, B, C), ref) in enumerate(zip(entries, refs)):
        assert_bit_exact(C, ref, f"layer slot {slot} ({bt.C5_SLOTS[slot]})")
    for p, *_ in plans.values():
        p.device_status()
        p.free()


@pytest.mark.parametrize("N", [128, 8])
def test_c3_integer_known_answer(N):
    """C3 (OPT-30B fc1 2:4, 28672 x 7168) on k_nm_mfma (col_direction_nm(32)), integer known
    answer bit for bit"""
    M, K = 28672, 7168
    row, col, _ = ds.two_four(M, K, 3)
    val = int_values(len(row), 9)
    plan = build(M, K, row, col, val, "col_direction_nm", 32, 1, N)
    info = plan.info()
    # 1,792 sixteen-row tiles: 256 workgroups of 7 (one per CU) below N = 128, 224 of 8 at N = 128
    assert info["device_kernel"] == "k_nm_mfma" and info["nm_tiles"] == (8 if N == 128 else 7), info
    B = int_B(K, N, 4)
    ref = exact_fp16(M, K, row, col, val, B)
    C = plan.spmm(B)
    torch.cuda.synchronize()
    assert_bit_exact(C, ref, f"C3 N={N}")
    plan.free()
