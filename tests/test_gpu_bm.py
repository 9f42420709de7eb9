"""GPU parity of k_mfma_bm / k_mfma_bm2 / k_mfma_kb (bitmap records, register-expanded matrix-core fragments):
every case against the oracle's SpMM of the same fp16 inputs (north_star fp16 tolerance),
the all-ones known answer bit-exactly, determinism of the K-split combine, replicas, and
the C2 shape against a torch fp32 dense product."""
import numpy as np
import pytest

import oracle_ffi as ofi

torch = pytest.importorskip("torch")
import generalsparse_amd as gsa  # noqa: E402
from generalsparse_amd import datasets as ds  # noqa: E402

from build_flags import experiments  # noqa: E402

pytestmark = [pytest.mark.gpu, experiments]
DEV = "cuda:0"


@pytest.fixture
def bm_on():
    old = {k: gsa.get_config(k) for k in ("MFMA_BM", "BM_SPLIT", "BM_WAVES", "MFMA_MAX_FILL", "BM_V2", "BM_KB")}
    gsa.set_config("MFMA_BM", 1)
    gsa.set_config("MFMA_MAX_FILL", 1 << 30)
    yield
    for k, v in old.items():
        gsa.set_config(k, v)


def cases():
    r, c, v = ds.pruned_weight(256, 512, 0.7, 13)
    yield "pruned", 256, 512, r, c, v
    r, c, v = ds.pruned_weight(1000, 3000, 0.8, 21)
    yield "pruned_ragged_M", 1000, 3000, r, c, v
    r, c, v = ds.pruned_weight(300, 4100, 0.5, 22)  # K not a multiple of 32
    yield "pruned_odd_K", 300, 4100, r, c, v
    keep = (r % 7) != 3  # empty rows inside row blocks
    yield "pruned_empty_rows", 300, 4100, r[keep], c[keep], v[keep]
    yield "dense_rows", 64, 200, *ds.random_rows(64, 200, 150.0, seed=3, empty_frac=0.0)


def run(M, K, row, col, val, p0, N, B=None, seed=0):
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", N, p0, 1).compile().upload("f16", 0)
    if B is None:
        B = np.random.default_rng(seed).uniform(-1, 1, (K, N)).astype(np.float16)
    C = plan.spmm(torch.from_numpy(B).to(DEV))
    torch.cuda.synchronize()
    return plan, C.float().cpu().numpy(), B


SHAPES = [(p0, N, split, waves) for p0 in (7, 40, 96) for N in (8, 16, 32, 64, 128) for split in (0, 3)
          for waves in (8,)] + [(p0, 32, split, waves) for p0 in (20, 80) for split in (0, 1, 3) for waves in (8, 4)]


KERNELS = ("k_mfma_bm", "k_mfma_bm2", "k_mfma_kb")


@pytest.mark.parametrize("variant", ["bm", "v2", "kb"])
@pytest.mark.parametrize("p0,N,split,waves", SHAPES)
def test_bm_matches_oracle(p0, N, split, waves, variant, bm_on):
    gsa.set_config("BM_SPLIT", split)
    gsa.set_config("BM_WAVES", waves)
    gsa.set_config("BM_V2", int(variant == "v2"))
    gsa.set_config("BM_KB", int(variant == "kb"))
    for case, M, K, row, col, val in cases():
        plan, C, B = run(M, K, row, col, val, p0, N)
        info = plan.info()
        assert info["device_kernel"] in KERNELS, (case, info)
        assert (info["device_kernel"] == "k_mfma_kb") == (variant == "kb"), (case, info)
        ref = ofi.spmm_ref(M, N, row, col, val.astype(np.float16).astype(np.float32), B.astype(np.float32), "f64")
        err = np.abs(C - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= 1e-1, (case, err.max())
        if split != 1:
            Bt = torch.from_numpy(B).to(DEV)
            np.testing.assert_array_equal(plan.spmm(Bt).float().cpu().numpy(), C)  # deterministic, counters re-armed
            plan.add_replica()
            np.testing.assert_array_equal(plan.spmm(Bt, replica=1).float().cpu().numpy(), C)
        plan.free()


@pytest.mark.parametrize("kb", [0, 1])
def test_bm_known_answer_and_c2(kb, bm_on):
    gsa.set_config("BM_KB", kb)
    M, K, N = 700, 9000, 32
    row, col, _ = ds.random_rows(M, K, 700.0, seed=8, empty_frac=0.1)  # row nnz < 2048: exact in fp16
    plan, C, _ = run(M, K, row, col, np.ones(len(row), np.float32), 64, N, B=np.ones((K, N), np.float16))
    assert plan.info()["device_kernel"] == ("k_mfma_kb" if kb else "k_mfma_bm")
    nnz_row = np.bincount(row.astype(np.int64), minlength=M).astype(np.float32)
    np.testing.assert_array_equal(C, np.repeat(nnz_row[:, None], N, axis=1))
    M = K = 5120
    r, c, v = ds.pruned_weight(M, K, 0.7, 13)
    A = torch.zeros((M, K), dtype=torch.float32)
    A[torch.from_numpy(r.astype(np.int64)), torch.from_numpy(c.astype(np.int64))] = torch.from_numpy(v).half().float()
    B = torch.randn((K, N), device=DEV, dtype=torch.float16)
    ref = A.to(DEV) @ B.float()
    for p0 in (80, 40):
        plan = gsa.Plan.from_coo(M, K, r, c, v).run_pipeline("block_total", N, p0, 1).compile().upload("f16", 0)
        info = plan.info()
        assert info["device_kernel"] == ("k_mfma_kb" if kb else "k_mfma_bm") and info["ksplit"] == 256 // (M // p0), info
        C = plan.spmm(B).float()
        err = ((C - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
        assert err <= 1e-1, err
        assert torch.equal(plan.spmm(B * 2).float(), 2 * C)  # linearity, deterministic
        plan.free()
