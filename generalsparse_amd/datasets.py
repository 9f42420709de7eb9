"""Synthetic, seeded stand-ins for the BASELINE.json configs.

The pruned OPT weights (Flash-LLM tooling) and SuiteSparse files are not
available offline; these generators reproduce the shapes, nnz and sparsity
structure with fixed seeds."""
import numpy as np


def pruned_weight(M, K, sparsity, seed):
    """Dense Gaussian M x K pruned to exactly round(sparsity*M*K) zeros by a
    global magnitude threshold (C2: 5120 x 5120, 70%, seed 13)."""
    rng = np.random.default_rng(seed)
    W = rng.standard_normal((M, K), dtype=np.float32)
    keep = int(round((1.0 - sparsity) * M * K))
    flat = np.abs(W).ravel()
    idx = np.argpartition(flat, flat.size - keep)[flat.size - keep:]
    idx.sort()
    row = (idx // K).astype(np.uint64)
    col = (idx % K).astype(np.uint64)
    val = W.ravel()[idx].astype(np.float32)
    return row, col, val


def two_four(M, K, seed):
    """2:4 structured by magnitude in each group of 4 along K (C3)."""
    rng = np.random.default_rng(seed)
    W = rng.standard_normal((M, K // 4, 4), dtype=np.float32)
    order = np.argsort(-np.abs(W), axis=2)[:, :, :2]
    order.sort(axis=2)
    g = np.arange(K // 4, dtype=np.int64)[None, :, None] * 4
    cols = (g + order).reshape(M, -1)
    vals = np.take_along_axis(W, order, axis=2).reshape(M, -1)
    row = np.repeat(np.arange(M, dtype=np.uint64), cols.shape[1])
    return row, cols.ravel().astype(np.uint64), vals.ravel().astype(np.float32)


def random_rows(M, K, mean_nnz_per_row, seed, empty_frac=0.0):
    """Uniform columns, Poisson row lengths (IG5-18 stand-in, C1)."""
    rng = np.random.default_rng(seed)
    lens = rng.poisson(mean_nnz_per_row, size=M)
    lens = np.minimum(lens, K)
    if empty_frac > 0:
        lens[rng.random(M) < empty_frac] = 0
    rows, cols = [], []
    for r in range(M):
        if lens[r]:
            c = np.sort(rng.choice(K, size=lens[r], replace=False))
            rows.append(np.full(lens[r], r, np.uint64))
            cols.append(c.astype(np.uint64))
    row = np.concatenate(rows) if rows else np.zeros(0, np.uint64)
    col = np.concatenate(cols) if cols else np.zeros(0, np.uint64)
    val = rng.uniform(-1, 1, size=len(row)).astype(np.float32)
    return row, col, val


def rmat(scale_n, nnz, seed, a=0.57, b=0.19, c=0.19, symmetric=False):
    """R-MAT power-law graph (C4 stand-ins), deduplicated, row-sorted."""
    rng = np.random.default_rng(seed)
    levels = int(np.ceil(np.log2(scale_n)))
    n = int((nnz // 2 if symmetric else nnz) * 1.3) + 1024  # symmetric: each sample gives 2 entries
    r = np.zeros(n, np.int64)
    cc = np.zeros(n, np.int64)
    for _ in range(levels):
        u = rng.random(n)
        down = u >= a + b
        right = ((u >= a) & (u < a + b)) | (u >= a + b + c)
        r = (r << 1) | down
        cc = (cc << 1) | right
    keep = (r < scale_n) & (cc < scale_n)
    r, cc = r[keep], cc[keep]
    if symmetric:
        r, cc = np.concatenate([r, cc]), np.concatenate([cc, r])
    key = np.unique(r * scale_n + cc)
    if len(key) > nnz:  # exact nnz: a seeded random subset (not the lowest rows)
        key = np.sort(rng.choice(key, size=nnz, replace=False))
    row = (key // scale_n).astype(np.uint64)
    col = (key % scale_n).astype(np.uint64)
    val = rng.uniform(-1, 1, size=len(row)).astype(np.float32)
    return row, col, val


def rmat_torch(scale_n, nnz, seed, device, a=0.57, b=0.19, c=0.19, symmetric=False):
    """The same R-MAT stand-in drawn with torch's generator on `device` (a GPU draws the
    234M-nnz com-Orkut stand-in in seconds where numpy takes minutes); deduplicated,
    row-sorted, exact nnz.  Returns numpy (row u64, col u64, val f32).  Not bit-identical
    to rmat() (different generator), same distribution."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    levels = int(np.ceil(np.log2(scale_n)))
    n = int((nnz // 2 if symmetric else nnz) * 1.3) + 1024
    r = torch.zeros(n, dtype=torch.int64, device=device)
    cc = torch.zeros(n, dtype=torch.int64, device=device)
    for _ in range(levels):
        u = torch.rand(n, generator=g, device=device)
        down = u >= a + b
        right = ((u >= a) & (u < a + b)) | (u >= a + b + c)
        r = (r << 1) | down.long()
        cc = (cc << 1) | right.long()
        del u, down, right
    keep = (r < scale_n) & (cc < scale_n)
    r, cc = r[keep], cc[keep]
    if symmetric:
        r, cc = torch.cat([r, cc]), torch.cat([cc, r])
    key = torch.unique(r * scale_n + cc)
    del r, cc
    if key.numel() > nnz:
        pick = torch.randperm(key.numel(), generator=g, device=device)[:nnz]
        key = torch.sort(key[pick]).values
    row = (key // scale_n).cpu().numpy().astype(np.uint64)
    col = (key % scale_n).cpu().numpy().astype(np.uint64)
    val = (torch.rand(key.numel(), generator=g, device=device) * 2 - 1).cpu().numpy().astype(np.float32)
    return row, col, val


def write_mtx(path, M, K, row, col, val=None):
    """Matrix Market coordinate file, 1-based, row-sorted, single spaces
    (what get_matrix_index_and_val_from_file parses, struct.cc:49-261)."""
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n")
        f.write(f"{M} {K} {len(row)}\n")
        if val is None:
            val = np.ones(len(row), np.float32)
        for s0 in range(0, len(row), 1 << 20):
            r = np.asarray(row[s0:s0 + (1 << 20)], np.int64) + 1
            c = np.asarray(col[s0:s0 + (1 << 20)], np.int64) + 1
            v = np.asarray(val[s0:s0 + (1 << 20)], np.float64)
            f.write("".join(f"{a} {b} {x:.6g}\n" for a, b, x in zip(r.tolist(), c.tolist(), v.tolist())))
