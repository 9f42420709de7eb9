"""Best-variant search over plans (the reference's obtain_result.py:6-67
scrapes the perf_result of every token_test pipeline and keeps the fastest).  Here each
candidate pipeline is built, uploaded and timed on the device with HIP events over rotated
replicas (no cache reuse), and the fastest plan is returned, optionally saved as a binary
plan file so later runs skip the search and the transforms.

This module is the one plan space of the product and of bench.py: the
candidate tables per matrix class (`CANDIDATES`, `candidates_for`) and per OPT layer shape
(`shape_candidates`), the config overrides a candidate carries while it is built
(`build_candidate`), and the search (`autotune`).  A candidate is (pipeline, p0, p1) or
(pipeline, p0, p1, {config key: value held while the plan is compiled and uploaded})."""
import math

# The canned plans per matrix class, each measured in profiles/ (DESIGN.md §4):
CANDIDATES = {
    # fp16 unstructured pruned weights (C2, OPT q_proj-like): k_mfma_ks row blocks with a K split
    # (block_total(40,1) KS_NT=1: 2 K ranges, A's groups by non-temporal loads -- the C2 winner,
    # profiles/r05n_nt3.txt), k_mfma_rows (tblock_warp_total(20,2)) and the gather families; at fp32
    # (the comparator's search) tblock_warp_total(24,2) on k_lds_rows_dma is the fastest (r06 ab_dma)
    "f16": [("block_total", 20, 1), ("block_total", 10, 1), ("block_total", 40, 1), ("block_total", 80, 1),
            ("block_total", 40, 1, {"KS_NT": 1}), ("block_total", 80, 1, {"KS_NT": 1}),
            ("tblock_warp_total", 20, 2), ("tblock_warp_total", 24, 2), ("tblock_warp_total", 4, 1),
            ("warp_segment", 4, 1), ("thread_total", 4, 1)],
    # fp16 2:4 structured (C3): the col-direction plan (32-nnz BMTs = 64-column k-steps) on the sparse
    # matrix cores; NM_NT (A's panel blocks by non-temporal loads) is the default, NM_TILES the
    # 16-row tiles per workgroup (0: the upload's rule)
    "f16_2to4": [("col_direction_nm", 32, 1), ("col_direction_nm", 32, 1, {"NM_NT": 0}),
                 ("col_direction_nm", 32, 1, {"NM_TILES": 8})],
    # fp32, short uniform rows (C1 IG5-18): token_test's default, row blocks and merge path
    "f32": [("thread_total", 4, 1), ("tblock_warp_total", 4, 1), ("tblock_warp_total", 32, 8),
            ("tblock_warp_total", 32, 16), ("tblock_warp_total", 64, 16), ("merge_path", 512, 1)],
    # fp32 power-law graphs (C4 webbase-1M): merge-path levels and the balanced / row-per-thread plans
    "f32_powerlaw": [("merge_path", 256, 1), ("merge_path", 512, 1), ("merge_path", 1024, 1),
                     ("balanced_block_total", 2048, 1), ("thread_total", 4, 1)],
    # over 50M nonzeros (com-Orkut): merge-path levels only (each plan is ~2 GB on the device and
    # minutes of host work; the balanced / row-per-thread plans are 4x-30x slower on C4)
    # (MP_COL_PARTS 4: the degree-ranked columns in 4 partitions, one pass each -- fabric reads 6.78x
    # -> 3.5x the algorithmic bytes at an even time, profiles/r06l_c4o_parts.txt)
    # (MP_COL_PARTS 2 at merge_path(2048): 1.90 against 1.97 ms unpartitioned, profiles/r06zq_c4o_parts.txt)
    "f32_powerlaw_large": [("merge_path", 512, 1), ("merge_path", 1024, 1), ("merge_path", 2048, 1),
                           ("merge_path", 1024, 1, {"MP_COL_PARTS": 4}), ("merge_path", 2048, 1, {"MP_COL_PARTS": 2})],
}
# plans that exist only in the fp32 form of a class: k_lds_rows_rs (fp32 at N = 32, BMWs of 5..8
# rows, one row per slot -- C2 fp32 29.4 us at (64,8) against 35.4 us for k_lds_rows_dma's (20,2),
# profiles/r06y_lds_rows_rs.txt); the fp32 comparator of an fp16 class searches these as well
F32_EXTRA = {"f16": [("tblock_warp_total", 64, 8), ("tblock_warp_total", 72, 8)]}
# the bench workloads (BASELINE.json configs) and the class each searches
WORKLOAD_CLASS = {"c1": "f32", "c2": "f16", "c3": "f16_2to4", "c4": "f32_powerlaw", "c4o": "f32_powerlaw_large"}


def row_block_rows(M, cus=256, max_rows=64):
    """BMTB height for the matrix-core row blocks (k_mfma_rows): the fewest whole rounds
    of one workgroup per CU, then the lowest height that keeps to that many rounds.  A
    workgroup streams all of B whatever its height, so a row block count just past a
    multiple of the CU count costs a whole extra round: 7168 rows in 20-row blocks are
    358 workgroups (two rounds on 256 CUs, 28.9 us on the C5 q/k/v/out shape), in 28-row
    blocks 256 (one round, 16.9 us); 28672 rows run best at 56 (two rounds).  MI355X:
    256 CUs (8 XCDs x 32)."""
    rounds = max(1, math.ceil(M / (cus * max_rows)))
    return max(1, math.ceil(M / (cus * rounds)))


def shape_candidates(M):
    """per-shape plans of the OPT layer weights (M rows) for the matrix-core kernels: KS_MIN_ROWS
    1000 keeps a block on k_mfma_rows; 56-row blocks of 7168-row shapes are 128 row blocks x 2 K
    ranges on k_mfma_ks; 112-row blocks are exactly 256 workgroups on every OPT-30B shape (7168
    rows: 64 blocks x 4 K ranges; fc1: 256 blocks x 1)"""
    rb = row_block_rows(M)
    return [("tblock_warp_total", rb, 2, {"KS_MIN_ROWS": 1000}), ("block_total", 56, 1, {}),
            ("block_total", 40, 1, {}), ("block_total", 80, 1, {}), ("block_total", 112, 1, {})]


def candidates_for(M, K, nnz, dtype, two_four=False, powerlaw=False):
    """the candidate list of a matrix: the class by value type and structure (2:4 panels,
    power-law rows, size), plus, for fp16 row blocks, the whole-CU-round k_mfma_rows height"""
    if dtype == "f16":
        if two_four:
            return list(CANDIDATES["f16_2to4"])
        c = list(CANDIDATES["f16"])
        rb = ("tblock_warp_total", row_block_rows(M), 2)
        if rb not in c:
            c.append(rb)
        return c
    if powerlaw:
        return list(CANDIDATES["f32_powerlaw_large" if nnz > 50_000_000 else "f32_powerlaw"])
    return list(CANDIDATES["f32"]) + [c for c in F32_EXTRA["f16"] if c not in CANDIDATES["f32"]]


def cand_key(c):
    """a candidate's label: pipeline(p0,p1) and its config overrides"""
    return "%s(%d,%d)%s" % (c[0], c[1], c[2], "".join(f" {a}={b}" for a, b in (c[3] if len(c) > 3 else {}).items()))


def build_candidate(M, K, row, col, val, cand, N, dtype, device=0):
    """the candidate's plan, compiled and uploaded with its config overrides held"""
    from . import Plan, get_config, set_config
    name, p0, p1 = cand[:3]
    over = cand[3] if len(cand) > 3 else {}
    old = {k: get_config(k) for k in over}
    try:
        for k, v in over.items():
            set_config(k, v)
        plan = Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile()
        plan.upload(dtype, device)
    finally:
        for k, v in old.items():
            set_config(k, v)
    return plan


def autotune(M, K, row, col, val, N, dtype="f16", candidates=None, device=0, reps=50, rotation_mb=640.0,
             save_path=None, two_four=False, powerlaw=False, rounds=3):
    """returns (best Plan (uploaded), {candidate key: kernel microseconds or error string}).
    Every candidate is timed in `rounds` interleaved rounds of `reps` rotated launches; its time
    is the median over the rounds (the chip's clock drifts from round to round)."""
    import torch
    from . import GsError
    tdt = torch.float16 if dtype == "f16" else torch.float32
    e = 2 if dtype == "f16" else 4
    dev = torch.device(f"cuda:{device}")
    if candidates is None:
        candidates = candidates_for(M, K, len(row), dtype, two_four=two_four, powerlaw=powerlaw)
    results, built = {}, []
    for cand in candidates:
        key = cand_key(cand)
        try:
            plan = build_candidate(M, K, row, col, val, cand, N, dtype, device)
        except GsError as ex:
            results[key] = str(ex)
            continue
        copies = max(2, int(math.ceil(rotation_mb * 1e6 / (plan.info()["device_bytes_A"] + K * N * e))))
        for _ in range(copies - 1):
            plan.add_replica()
        Bs = [torch.randn((K, N), device=dev, dtype=tdt) for _ in range(copies)]
        Cs = [torch.empty((M, N), device=dev, dtype=tdt) for _ in range(copies)]
        built.append([key, plan, plan.rotation(Bs, Cs), Bs, Cs, []])
    for _ in range(max(1, rounds)):
        for b in built:
            rot = b[2]
            rot.run(5, 0)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rot.run(reps, 0)
            e1.record()
            torch.cuda.synchronize(dev)
            b[5].append(e0.elapsed_time(e1) / reps * 1e3)
    best = None
    for b in built:
        us = sorted(b[5])[len(b[5]) // 2]
        results[b[0]] = round(us, 3)
        if best is None or us < best[0]:
            best = (us, b)
    if best is None:
        raise GsError("no candidate plan could be built")
    for b in built:
        b[2] = b[3] = b[4] = None
        if b is not best[1]:
            b[1].free()
    plan = best[1][1]
    if save_path:
        plan.save(save_path)
    return plan, results
