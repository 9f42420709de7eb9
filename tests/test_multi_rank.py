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
    import bench
    batch = [bench.C5_SLOTS[s] for _ in range(48) for s in range(len(bench.C5_SLOTS))]
    sizes = [int(round(0.2 * m * n)) for m, n in (bench.C5_SHAPES[k] for k in batch)]
    assert sum(sizes) == 48 * (4 * 10276045 + 2 * 41104179)
    for world in (1, 2, 4, 8):
        owner, load = bench.lpt_assign(sizes, world)
        assert len(owner) == 288 and set(owner) == set(range(world))
        assert max(load) / min(load) <= 1.02
