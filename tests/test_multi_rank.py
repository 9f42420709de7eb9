"""The N>1 bench path on CPU ranks (gloo, world_size 2): each rank builds the plan
of its own shard (row-sharded batch of independent matrices, no data-path
exchange), the job time is the max over ranks, and the whole-job value counts
every rank's work (bench.py's helpers, the ones the GPU run uses)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import generalsparse_amd as gsa
    from generalsparse_amd import datasets as ds
    M = K = 256
    row, col, val = ds.pruned_weight(M, K, 0.7, bench.shard_seed(rank))
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline("block_total", 32, 20, 1).compile()
    first = plan.array("TBLOCK_META_first_row_indices_0")
    wall = 1.0 + rank  # rank 1 is the slow one
    job = bench.max_over_ranks(wall, dist, torch)
    value = bench.whole_job_gflops(world, 2.0 * len(row) * 32, 10, job)
    digest = torch.tensor([float(np.sum(col[:100]))])
    gathered = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(gathered, digest)
    out[rank] = (job, value, len(first), [g.item() for g in gathered])
    dist.barrier()
    dist.destroy_process_group()


def test_two_gloo_ranks_shard_and_max_time():
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_rank_main, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    (j0, v0, n0, g0), (j1, v1, n1, g1) = res[0], res[1]
    assert j0 == j1 == 2.0                       # max over ranks
    assert v0 == v1                              # same job value on every rank
    assert n0 == n1 == 256 // 20 + 2             # ceil(256/20) BMTBs + 1
    assert g0[0] != g0[1]                        # each rank built its own shard


def test_c5_lpt_split_is_balanced():
    """C5 batch (48 OPT-30B layers): LPT on nnz gives every rank the same share at
    1, 2, 4 and 8 ranks (balance within 2%)"""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from generalsparse_amd import batch as bt
    for world in (1, 2, 4, 8):
        batch, owner, load = bt.c5_assignment(48, world)
        sizes = [bt.nnz_of_shape(b[2]) for b in batch]
        assert sum(sizes) == 48 * (4 * 10276045 + 2 * 41104179)
        assert len(owner) == 288 and set(owner) == set(range(world))
        assert max(load) / min(load) <= 1.02


def _c5_main(rank, world, port, layers, out):
    """run_c5's per-rank part without the GPU: the assignment every rank computes on its
    own, its launch sequence, and the job nnz gathered over the ranks"""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from generalsparse_amd import batch as bt
    batch, owner, load = bt.c5_assignment(layers, world)
    seq = bt.rank_sequence(batch, owner, rank)
    mine = torch.tensor([float(sum(bt.nnz_of_shape(s[2]) for s in seq))], dtype=torch.float64)
    allv = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allv, mine)
    out[rank] = (seq, [v.item() for v in allv], owner)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("layers", [2, 48])
def test_c5_batch_sequence_two_gloo_ranks(layers):
    """the C5 batch over 2 gloo ranks: both ranks compute the same LPT assignment, their
    launch sequences cover every matrix of the batch exactly once in layer order, replica
    k of a shape is that shape's k-th instance on the rank, and the gathered per-rank nnz
    add up to the batch (bench.py run_c5's assignment and sequencing)"""
    sys.path.insert(0, ROOT)
    from generalsparse_amd import batch as bt
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_c5_main, args=(2, port, layers, out), nprocs=2, join=True)
        res = dict(out)
    assert res[0][2] == res[1][2]                         # one assignment, computed twice
    covered = sorted((l, s) for r in (0, 1) for (l, s, _, _) in res[r][0])
    assert covered == [(l, s) for l in range(layers) for s in range(6)]
    for r in (0, 1):
        seq = res[r][0]
        assert [(l, s) for (l, s, _, _) in seq] == sorted((l, s) for (l, s, _, _) in seq)
        for shape in bt.C5_SHAPES:
            reps = [k for (_, _, sh, k) in seq if sh == shape]
            assert reps == list(range(len(reps)))
    total = sum(bt.nnz_of_shape(b[2]) for b in bt.c5_batch(layers))
    assert res[0][1] == res[1][1] and sum(res[0][1]) == total
    assert max(res[0][1]) / min(res[0][1]) <= (1.02 if layers == 48 else 1.5)


def _hip_spmm(M, K, N, row, col, val, B, dtype, pipeline, p0):
    """C = A B through the HIP library on cuda:0 (a gs plan of the shard's COO), on the host"""
    import generalsparse_amd as gsa
    plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipeline, N, p0, 1).compile().upload(dtype, 0)
    tdt = torch.float16 if dtype == "f16" else torch.float32
    C = plan.spmm(torch.from_numpy(B).to("cuda:0", tdt))
    torch.cuda.synchronize()
    out = C.cpu()
    plan.free()
    return out


def _shard_main(rank, world, port, mode, out, hip=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_ffi as ofi
    from generalsparse_amd import datasets as ds
    from generalsparse_amd import shard as sd
    M, N = 3000, 8
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 6, M)
    lens[100] = 4000                      # a row longer than a shard: split over ranks
    lens[-50:] = 0                        # trailing empty rows
    row = np.repeat(np.arange(M, dtype=np.uint64), lens)
    col = rng.integers(0, 500, len(row)).astype(np.uint64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    B = rng.uniform(-1, 1, (500, N)).astype(np.float32)
    shards = (sd.nnz_exact_shards if mode == "nnz" else sd.balanced_row_shards)(row, M, world)
    sh = shards[rank]
    m, r, c, v = sd.local_coo(row, col, val, sh)
    if hip:
        # the GPU path: the shard's plan (fp16 for nnz shards, fp32 for row shards) on the
        # HIP library; the fp32 edge partials from a 2-row fp32 side plan, as bench.py does
        dt = "f16" if mode == "nnz" else "f32"
        Bx = B.astype(np.float16).astype(np.float32) if dt == "f16" else B
        C_local = _hip_spmm(m, 500, N, r, c, v, Bx, dt, "merge_path", 64) if m else torch.zeros((0, N))
    else:
        C_local = torch.from_numpy(ofi.spmm_ref(m, N, r, c, v, B, "f64").astype(np.float32)) if m else torch.zeros((0, N))
    edges = None
    if mode == "nnz" and m:
        er, ec, ev = sd.edge_rows(row, col, val, sh)
        if hip:
            edges = _hip_spmm(2, 500, N, er, ec, ev, B.astype(np.float16).astype(np.float32), "f32", "merge_path", 64)
        else:
            edges = torch.from_numpy(ofi.spmm_ref(2, N, er, ec, ev, B, "f64").astype(np.float32))
            C_local = C_local.half()   # an fp16 plan's output; the split rows use the fp32 edge partials
    first = sd.combine_boundaries(C_local, shards, rank, dist, torch, edges) if mode == "nnz" else 0
    C_local = C_local.float()
    out[rank] = (sh.row_lo + first, C_local[first:].numpy().copy(), sh.z1 - sh.z0)
    dist.barrier()
    dist.destroy_process_group()


def _check_shards(mode, world, hip):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as ofi
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_shard_main, args=(world, port, mode, out, hip), nprocs=world, join=True)
        res = dict(out)
    M, N = 3000, 8
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 6, M)
    lens[100] = 4000
    lens[-50:] = 0
    row = np.repeat(np.arange(M, dtype=np.uint64), lens)
    col = rng.integers(0, 500, len(row)).astype(np.uint64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    B = rng.uniform(-1, 1, (500, N)).astype(np.float32)
    if hip and mode == "nnz":
        B = B.astype(np.float16).astype(np.float32)   # the fp16 plan's B
    ref = ofi.spmm_ref(M, N, row, col, val, B, "f64")
    got = np.zeros((M, N))
    seen = np.zeros(M, int)
    for r in range(world):
        lo, blk, nz = res[r]
        got[lo:lo + len(blk)] = blk
        seen[lo:lo + len(blk)] += 1
    assert sum(res[r][2] for r in range(world)) == len(row)
    held = seen > 0
    assert (seen <= 1).all()
    tol = 1e-3 if mode == "nnz" else 1e-5   # nnz mode: fp16 rows, split rows rounded once after the fp32 sum
    if hip and mode == "nnz":
        tol = 4e-3                           # fp16 values of the plan; fp32 accumulation on the device
    np.testing.assert_allclose(got[held], ref[held], rtol=tol, atol=tol)
    if mode == "nnz" and not hip:
        long_row = got[100]    # split over every rank: exactly the fp16 rounding of the fp32 sum
        np.testing.assert_array_equal(long_row, ref[100].astype(np.float32).astype(np.float16).astype(np.float64))
    # rows no rank holds are the trailing empty rows (zero in the full product)
    assert np.all(ref[~held] == 0)


@pytest.mark.parametrize("mode", ["rows", "nnz"])
@pytest.mark.parametrize("world", [2, 3])
def test_single_matrix_shards_combine_to_full_spmm(mode, world):
    """one matrix over `world` gloo ranks: balanced row ranges (no exchange) or
    nnz-exact ranges (split rows combined by one all-reduce), reassembled rows equal
    the unsharded oracle SpMM"""
    _check_shards(mode, world, hip=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["rows", "nnz"])
def test_single_matrix_shards_hip_local_spmm(mode):
    """the same over two gloo ranks whose local SpMM (and fp32 edge partials) run on the
    HIP library on cuda:0 -- the product path of every rank, combined on the host"""
    _check_shards(mode, 2, hip=True)


def test_row_block_rows_fill_whole_cu_rounds():
    """matrix-core BMTB heights: whole rounds of one workgroup per CU (256 on MI355X) at
    the lowest height, at most 64 rows (C2 keeps 20; the C5 shapes get 28 / 56)"""
    import math
    from generalsparse_amd.autotune import row_block_rows
    from generalsparse_amd import batch as bt
    assert row_block_rows(5120) == 20
    assert {k: bt.shape_pipeline(k)[1] for k in bt.C5_SHAPES} == {"attn": 28, "fc1": 56, "fc2": 28}
    for M in (1, 255, 256, 257, 5120, 7168, 16385, 28672, 100000):
        r = row_block_rows(M)
        assert 1 <= r <= 64
        rounds = math.ceil(math.ceil(M / r) / 256)
        assert rounds == max(1, math.ceil(M / (256 * 64)))
        assert r == 1 or math.ceil(math.ceil(M / (r - 1)) / 256) > rounds


def test_bench_searches_the_product_plan_space():
    """bench.py keeps no candidate table of its own; every workload searches
    autotune.CANDIDATES through WORKLOAD_CLASS, and the C5 shapes autotune.shape_candidates"""
    import os
    from generalsparse_amd import autotune as at
    from generalsparse_amd import batch as bt
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    assert "CANDIDATES = [" not in src and "CANDIDATES_C" not in src
    for wl in ("c1", "c2", "c3", "c4", "c4o"):
        assert f'at.WORKLOAD_CLASS["{wl}"]' in src
        assert at.CANDIDATES[at.WORKLOAD_CLASS[wl]]
    assert ("block_total", 40, 1, {"KS_NT": 1}) in at.CANDIDATES["f16"]
    assert bt.shape_candidates("fc1") == at.shape_candidates(28672)
    assert at.candidates_for(5120, 5120, 7864320, "f16")[:len(at.CANDIDATES["f16"])] == at.CANDIDATES["f16"]
    assert at.candidates_for(28672, 7168, 1, "f16", two_four=True) == at.CANDIDATES["f16_2to4"]
    assert at.candidates_for(1, 1, 234_000_000, "f32", powerlaw=True) == at.CANDIDATES["f32_powerlaw_large"]
