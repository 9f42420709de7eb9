"""The C5 batch (BASELINE.json configs[4]): every pruned weight of OPT-30B's 48
decoder layers -- per layer q, k, v, out (7168 x 7168), fc1 (28672 x 7168) and fc2
(7168 x 28672), 80% unstructured, fp16, N = 32 -- split over the ranks of one node.

SURVEY.md §8e: the matrices are independent, so the batch shards by whole matrices
(longest-processing-time greedy on nnz, no data-path collective); each rank runs its
share of SpMMs per step.  The assignment and the per-rank launch sequence are pure
Python (tested with gloo ranks on the CPU); `build_rank_batch` puts one seeded matrix
per shape on the rank's GPU with one plan replica per batch instance, so every
instance streams its own HBM copy of A."""

C5_SHAPES = {"attn": (7168, 7168), "fc1": (28672, 7168), "fc2": (7168, 28672)}
C5_SLOTS = ["attn", "attn", "attn", "attn", "fc1", "fc2"]
C5_SPARSITY = 0.8


def lpt_assign(sizes, world):
    """longest-processing-time greedy: item i -> rank, ties to the lowest rank"""
    load = [0] * world
    owner = [0] * len(sizes)
    for i in sorted(range(len(sizes)), key=lambda i: -sizes[i]):
        r = min(range(world), key=lambda r: load[r])
        owner[i] = r
        load[r] += sizes[i]
    return owner, load


def nnz_of_shape(shape, sparsity=C5_SPARSITY):
    m, n = C5_SHAPES[shape]
    return int(round((1 - sparsity) * m * n))


def c5_batch(layers):
    """the batch in layer order: (layer, slot index, shape name)"""
    return [(l, s, C5_SLOTS[s]) for l in range(layers) for s in range(len(C5_SLOTS))]


def c5_assignment(layers, world):
    """(batch, owner, load): the LPT split of the batch's matrices over `world` ranks"""
    batch = c5_batch(layers)
    owner, load = lpt_assign([nnz_of_shape(b[2]) for b in batch], world)
    return batch, owner, load


def rank_sequence(batch, owner, rank):
    """this rank's launches in batch order: (layer, slot, shape, replica); replica k of a
    shape = the k-th instance of that shape on this rank"""
    seq, rep = [], {}
    for b, o in zip(batch, owner):
        if o != rank:
            continue
        k = rep.get(b[2], 0)
        seq.append((b[0], b[1], b[2], k))
        rep[b[2]] = k + 1
    return seq


def shape_seed(rank, shape):
    """one distinct seeded matrix per shape per rank"""
    return 1000 + 8 * rank + list(C5_SHAPES).index(shape)


def shape_pipeline(shape):
    """the pipeline of a shape's plan: BMTB row blocks sized to whole CU rounds
    (autotune.row_block_rows: 28 rows for the 7168-row shapes, 56 for fc1)"""
    from .autotune import row_block_rows
    return ("tblock_warp_total", row_block_rows(C5_SHAPES[shape][0]), 2)


def shape_candidates(shape):
    """per-shape plan candidates for the matrix-core kernels (bench.py searches them for the
    headline layer): autotune.shape_candidates of the shape's row count"""
    from .autotune import shape_candidates as sc
    return sc(C5_SHAPES[shape][0])


def build_plan(gsa, m, n, row, col, val, N, cand, local):
    """a shape's plan from a candidate (pipeline, p0, p1[, config overrides]): autotune.build_candidate"""
    from .autotune import build_candidate
    return build_candidate(m, n, row, col, val, cand, N, "f16", local)


def build_rank_batch(seq, rank, N, gsa, ds, torch, dev, local, pipeline=None, keep_coo=False,
                     sparsity=C5_SPARSITY, choice=None):
    """plans (one per shape, one replica per instance), B and C buffers (two per shape,
    alternating), and the launch list [(plan, replica, B, C, shape)].  `pipeline`
    (name, p0, p1) overrides the per-shape choice of shape_pipeline; `choice` maps a
    shape to a shape_candidates entry."""
    count = {}
    for (_, _, k, _) in seq:
        count[k] = count.get(k, 0) + 1
    plans, Bs, Cs, coo = {}, {}, {}, {}
    for k, (m, n) in C5_SHAPES.items():
        if not count.get(k):
            continue
        row, col, val = ds.pruned_weight(m, n, sparsity, shape_seed(rank, k))
        pl = pipeline or (choice or {}).get(k) or shape_pipeline(k)
        plan = build_plan(gsa, m, n, row, col, val, N, pl, local)
        for _ in range(count[k] - 1):
            plan.add_replica()
        plans[k] = plan
        g = torch.Generator(device=dev)
        g.manual_seed(7 + shape_seed(rank, k))
        Bs[k] = [torch.rand((n, N), device=dev, generator=g).mul_(2).sub_(1).half() for _ in range(2)]
        Cs[k] = [torch.empty((m, N), device=dev, dtype=torch.float16) for _ in range(2)]
        if keep_coo:
            coo[k] = (row, col, val)
        del row, col, val
    launches = []
    for i, (_, _, k, r) in enumerate(seq):
        launches.append((plans[k], r, Bs[k][i % 2], Cs[k][i % 2], k))
    return plans, launches, coo
