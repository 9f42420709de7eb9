"""Best-variant search over plans (the reference's obtain_result.py
scrapes the perf_result of every token_test pipeline and keeps the fastest).  Here each
candidate pipeline is built, uploaded and timed on the device with HIP events over rotated
replicas (no cache reuse), and the fastest plan is returned, optionally saved as a binary
plan file so later runs skip the search and the transforms."""
import math

from . import Plan, GsError

# the canned pipelines worth trying, by value type (fp16 plans may reach the matrix cores)
DEFAULT_CANDIDATES = {
    "f16": [("tblock_warp_total", 20, 2), ("block_total", 20, 1), ("col_direction_nm", 32, 1),
            ("merge_path", 512, 1), ("thread_total", 4, 1), ("warp_segment", 4, 1)],
    "f32": [("merge_path", 512, 1), ("thread_total", 4, 1), ("tblock_warp_total", 4, 1),
            ("warp_bit_map_interleaved", 4, 1), ("balanced_warp_total", 256, 1)],
}


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


def autotune(M, K, row, col, val, N, dtype="f16", candidates=None, device=0, reps=50, rotation_mb=640.0,
             save_path=None):
    """returns (best Plan (uploaded), {variant: kernel microseconds or error string})"""
    import torch
    tdt = torch.float16 if dtype == "f16" else torch.float32
    e = 2 if dtype == "f16" else 4
    dev = torch.device(f"cuda:{device}")
    results, best = {}, None
    if candidates is None:
        candidates = list(DEFAULT_CANDIDATES[dtype])
        if dtype == "f16" and ("tblock_warp_total", row_block_rows(M), 2) not in candidates:
            candidates.insert(0, ("tblock_warp_total", row_block_rows(M), 2))
    for name, p0, p1 in candidates:
        key = f"{name}({p0},{p1})"
        try:
            plan = Plan.from_coo(M, K, row, col, val).run_pipeline(name, N, p0, p1).compile().upload(dtype, device)
        except GsError as ex:
            results[key] = str(ex)
            continue
        copies = max(2, int(math.ceil(rotation_mb * 1e6 / (plan.info()["device_bytes_A"] + K * N * e))))
        for _ in range(copies - 1):
            plan.add_replica()
        Bs = [torch.randn((K, N), device=dev, dtype=tdt) for _ in range(copies)]
        Cs = [torch.empty((M, N), device=dev, dtype=tdt) for _ in range(copies)]
        rot = plan.rotation(Bs, Cs)
        rot.run(5, 0)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rot.run(reps, 0)
        e1.record()
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) / reps * 1e3
        results[key] = round(us, 3)
        del Bs, Cs, rot
        if best is None or us < best[0]:
            if best is not None:
                best[2].free()
            best = (us, key, plan)
        else:
            plan.free()
    if best is None:
        raise GsError("no candidate plan could be built")
    plan = best[2]
    if save_path:
        plan.save(save_path)
    return plan, results
