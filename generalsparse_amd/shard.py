"""One matrix split across GPUs, one process per GPU.

Two partitions of the row-sorted COO of A:

- ``balanced_row_shards``: contiguous row ranges with about equal nnz, cut by the
  balanced-interval rule (get_begin_rows_of_child_after_balance_blocking_in_row_direction,
  data_transform_common.cc:960-989) with nnz_per_interval = ceil(nnz / world).  Rows are
  never split, C rows are disjoint, there is no exchange.
- ``nnz_exact_shards``: rank r takes nonzeros [r*nnz/world, (r+1)*nnz/world) (the merge-path
  level rule at work_size = nnz/world, nonzeros only).  A row can be split between ranks;
  ``combine_boundaries`` is the exchange step: every rank publishes the partial sum of its
  first row in its own slot of a small world x N buffer, one all-reduce (SUM; RCCL over xGMI
  on GPU ranks, gloo on CPU ranks) gathers them, and the rank where a split row starts adds
  the other ranks' partials in rank order (deterministic).

Each rank builds the plan of its local sub-matrix (rows relative to its first row), so its C
is the block of rows [row_lo, row_hi] of the full C.
"""
from dataclasses import dataclass

import numpy as np


@dataclass
class Shard:
    rank: int
    z0: int          # first nonzero (row-sorted order)
    z1: int          # one past the last
    row_lo: int      # first output row held (inclusive)
    row_hi: int      # last output row held (inclusive); row_hi < row_lo: no rows
    owns_first: bool  # the shard's first row starts in it (it stores that row)


def _shards_from_nz_cuts(row, M, cuts):
    out = []
    world = len(cuts) - 1
    for r in range(world):
        z0, z1 = int(cuts[r]), int(cuts[r + 1])
        if z1 > z0:
            lo, hi = int(row[z0]), int(row[z1 - 1])
            owns = z0 == 0 or int(row[z0 - 1]) != lo
        else:
            lo, hi, owns = 0, -1, False
        out.append(Shard(r, z0, z1, lo, hi, owns))
    return out


def balanced_row_shards(row, M, world):
    """rows never split; empty rows stay with the shard before them (the first shard
    also takes the leading empty rows)"""
    row = np.asarray(row, dtype=np.int64)
    nnz = len(row)
    per = max(1, -(-nnz // world))
    cnt = np.bincount(row, minlength=M)
    acc = np.cumsum(cnt)
    cuts_rows = [0]
    c = 0
    for i in range(M):  # data_transform_common.cc:960-989 with nnz_per_interval = per
        c += cnt[i]
        if c >= per and len(cuts_rows) < world:
            cuts_rows.append(i + 1)
            c = 0
    while len(cuts_rows) < world + 1:
        cuts_rows.append(M)
    cuts_rows[-1] = M
    out = []
    for r in range(world):
        a, b = cuts_rows[r], cuts_rows[r + 1]
        z0 = int(acc[a - 1]) if a > 0 else 0
        z1 = int(acc[b - 1]) if b > 0 else 0
        out.append(Shard(r, z0, z1, a, b - 1, True))
    return out


def nnz_exact_shards(row, M, world):
    nnz = len(row)
    cuts = [r * nnz // world for r in range(world + 1)]
    return _shards_from_nz_cuts(np.asarray(row), M, cuts)


def local_coo(row, col, val, sh):
    """the shard's sub-matrix: (rows held, row indices relative to row_lo, cols, vals)"""
    if sh.row_hi < sh.row_lo:
        return 0, row[:0], col[:0], val[:0]
    r = np.asarray(row[sh.z0:sh.z1], dtype=np.uint64) - np.uint64(sh.row_lo)
    return sh.row_hi - sh.row_lo + 1, r, col[sh.z0:sh.z1], val[sh.z0:sh.z1]


def edge_rows(row, col, val, sh):
    """the shard's first and last row as a 2-row COO (rows 0 and 1; the same row twice when
    the shard holds one row): the rows a nnz-exact split can share with other ranks"""
    if sh.row_hi < sh.row_lo:
        return None
    r = np.asarray(row[sh.z0:sh.z1], dtype=np.int64)
    first = r == sh.row_lo
    last = r == sh.row_hi
    rr = np.concatenate([np.zeros(first.sum(), np.uint64), np.ones(last.sum(), np.uint64)])
    cc = np.concatenate([col[sh.z0:sh.z1][first], col[sh.z0:sh.z1][last]])
    vv = np.concatenate([val[sh.z0:sh.z1][first], val[sh.z0:sh.z1][last]])
    return rr, cc, vv


def combine_boundaries(C_local, shards, rank, dist, torch, edges_fp32=None):
    """nnz-exact shards: the exchange step.  Every rank publishes the partial of its
    first row in its slot of a world x N buffer; one all-reduce (SUM, one writer per
    slot) gathers them; a rank whose last row continues into later ranks (it starts
    that row) adds their partials in rank order.  C_local: (rows held, N) tensor on
    this rank's device, rows [row_lo, row_hi] of C.  edges_fp32: optional (2, N) fp32
    partials of the shard's first and last rows (e.g. from a 2-row fp32 side plan over
    ``edge_rows``), so fp16 plans round a split row once, after the sum; without it the
    partials are read from C_local.  Returns the index of the first complete row of
    C_local (1 when another rank starts our first row)."""
    world = len(shards)
    sh = shards[rank]
    has = sh.row_hi >= sh.row_lo
    buf = torch.zeros((world, C_local.shape[1]), dtype=torch.float32, device=C_local.device)
    first = edges_fp32[0] if edges_fp32 is not None else (C_local[0].float() if has else None)
    last = edges_fp32[1] if edges_fp32 is not None else (C_local[-1].float() if has else None)
    if has:
        buf[rank] = first
    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
    if has and (sh.owns_first or sh.row_hi != sh.row_lo):
        acc = last.clone()
        for q in range(rank + 1, world):
            s = shards[q]
            if s.row_hi < s.row_lo or s.row_lo != sh.row_hi:
                break
            acc = acc + buf[q]
            if s.row_hi != s.row_lo:
                break  # the row closes in rank q
        C_local[-1] = acc.to(C_local.dtype)
    return 1 if has and not sh.owns_first else 0
