#!/usr/bin/env python3
"""SpMM benchmark (BASELINE.json metric: SpMM GFLOP/s + achieved HBM GB/s vs
rocSPARSE, pruned-weight fp16 N=32).

N=1 workload (configs[1]): OPT-13B q_proj stand-in, 5120 x 5120, 70% unstructured
(global magnitude pruning of a seeded Gaussian, nnz 7,864,320), fp16 A/B/C, fp32
accumulation, dense N = 32.  A "step" = one SpMM of one matrix.  Inputs are resident
in HBM; every step uses the next of R independent device copies of A (and B), R sized
on the bytes the selected kernel reads so the rotation set exceeds 512 MB and the
256 MB Infinity Cache cannot serve A (SURVEY.md §8d "cache honesty").  The plan is
chosen first (the reference's best-variant search, obtain_result.py): every candidate
pipeline is timed over `--search-reps` launches; then the chosen plan runs W untimed
warm-up steps and exactly K timed steps between barriers and device syncs.

Multi-GPU (`--gpus N`, N > 1): one process per GPU.  Started without WORLD_SIZE,
bench.py launches the N ranks itself (torch.distributed.run on 127.0.0.1) before
anything touches a GPU.  The default N > 1 workload is configs[4] (C5): the 288
matrices of the 48-layer OPT-30B 80%-pruned batch split over the ranks by LPT on nnz
(strong scaling, no data-path collective).  `--workload c2` keeps the weak-scaling
batch of one C2 matrix per rank.  The time is the max over ranks.

--workload c1 | c3 | c4 | c4o | c5 measures the other BASELINE.json configs; c5h the
north_star headline (one OPT-30B layer at 70%, with rocSPARSE per shape).

Prints one JSON line on rank 0."""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=500)  # clocks settle over the first ~1000 launches
    ap.add_argument("--pipeline", default="auto",
                    help="plan pipeline, or 'auto' = best of the candidates (obtain_result.py takes the max)")
    ap.add_argument("--rotation-mb", type=float, default=640.0)
    ap.add_argument("--no-rocsparse", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-north-star", action="store_true",
                    help="c2: skip the north_star object (the OPT-30B 70% layer timed in the same run)")
    ap.add_argument("--p0", type=int, default=None, help="with --pipeline: run only this plan parameter")
    ap.add_argument("--p1", type=int, default=None)
    ap.add_argument("--workload", choices=("c1", "c2", "c3", "c4", "c4o", "c5", "c5h"), default=None,
                    help="default: c2 on one GPU, c5 (the sharded batch) on several")
    ap.add_argument("--search-reps", type=int, default=100, help="launches per candidate plan in the plan search")
    ap.add_argument("--search-rounds", type=int, default=3,
                    help="interleaved timing rounds per candidate plan (the median decides)")
    ap.add_argument("--n-sweep", default="", help="also time the chosen plan family at these dense widths, e.g. 8,32,128")
    ap.add_argument("--layers", type=int, default=48, help="c5: OPT-30B layers in the batch")
    ap.add_argument("--group", type=int, default=-1,
                    help="c5/c5h: 1 = the batch through gs_spmm_batch (grouped k_mfma_ks launches, dealt over "
                         "--streams), 0 = one launch per matrix over --streams streams; -1 = the measured best: "
                         "c5h grouped on one stream (57.2 vs 54.9 TFLOP/s), c5 per matrix over two streams (61.7 vs "
                         "58.7-60.0; profiles/r04g_*)")
    ap.add_argument("--streams", type=int, default=-1,
                    help="c5/c5h: HIP streams the batch's launches rotate over (2: one launch's tail overlaps the "
                         "next one's start; profiles/r03_c5_streams.json); -1 = as --group -1 picks")
    ap.add_argument("--shard", choices=("batch", "rows", "nnz"), default="batch",
                    help="c4/c4o with N>1: batch = a matrix per rank (weak); rows / nnz = one matrix split "
                         "over the ranks (strong; nnz splits rows and combines them with one all-reduce)")
    ap.add_argument("--M", type=int, default=0)
    ap.add_argument("--K", type=int, default=0)
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--sparsity", type=float, default=0.7)
    ap.add_argument("--config", action="append", default=[], metavar="KEY=INT",
                    help="engine switch (gs_set_config_int), e.g. BM_VARIANT=1; repeatable")
    return ap.parse_args()


def resolve_workload(a, world):
    if a.workload is None:
        a.workload = "c5" if world > 1 else "c2"
    if a.group < 0:
        a.group = 1 if a.workload == "c5h" else 0
    if a.streams < 0:
        a.streams = 1 if a.workload == "c5h" else 2
    dflt = {"c1": (47894, 41550, 8), "c2": (5120, 5120, 32), "c3": (28672, 7168, 128), "c4": (1000005, 1000005, 8),
            "c4o": (3072441, 3072441, 8), "c5": (7168, 7168, 32), "c5h": (7168, 7168, 32)}[a.workload]
    a.M, a.K, a.N = a.M or dflt[0], a.K or dflt[1], a.N or dflt[2]


def launch_ranks(n):
    """--gpus N without a launcher: start N ranks (one per GPU) with torch.distributed.run
    and exit with its status.  Nothing here touches a GPU."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


WORKLOADS = {
    "c2": {"metric": "SpMM GFLOP/s + achieved HBM GB/s vs rocSPARSE, pruned-weight fp16 N=32",
           "workload": "OPT-13B q_proj stand-in {M}x{K} 70% unstructured, fp16, N={N}",
           "data": "synthetic (seeded magnitude-pruned Gaussian)"},
    "c3": {"metric": "SpMM GFLOP/s + achieved HBM GB/s vs rocSPARSE, 2:4 pruned-weight fp16 N=128 (configs[2])",
           "workload": "OPT-30B fc1 stand-in {M}x{K} 2:4 structured, fp16, N={N}",
           "data": "synthetic (seeded Gaussian, 2:4 magnitude pruning per group of 4)", "dtype": "f16"},
    "c1": {"metric": "SpMM GFLOP/s (configs[0], IG5-18 stand-in; the reference runs it on the CPU only)",
           "workload": "IG5-18 stand-in {M}x{K} nnz~1.79M, Poisson rows (mean 37.4), fp32, N={N}",
           "data": "synthetic (seeded uniform columns, Poisson row lengths; the .mtx is not available offline)",
           "dtype": "f32"},
    "c4": {"metric": "SpMM GFLOP/s + achieved HBM GB/s vs rocSPARSE, power-law fp32 N=8 (configs[3], webbase-1M)",
           "workload": "webbase-1M stand-in {M}x{K} nnz 3105536 R-MAT(.57,.19,.19), fp32, N={N}",
           "data": "synthetic (seeded R-MAT, deduplicated, row-sorted; SuiteSparse files are not available offline)",
           "dtype": "f32", "nnz": 3105536, "seed": 1, "symmetric": False},
    "c4o": {"metric": "SpMM GFLOP/s + achieved HBM GB/s vs rocSPARSE, power-law fp32 N=8 (configs[3], com-Orkut)",
            "workload": "com-Orkut stand-in {M}x{K} nnz 234370166 symmetric R-MAT(.57,.19,.19), fp32, N={N}",
            "data": "synthetic (seeded R-MAT, symmetrised, deduplicated, row-sorted)",
            "dtype": "f32", "nnz": 234370166, "seed": 2, "symmetric": True},
}
WORKLOADS["c2"]["dtype"] = "f16"


# The plan candidates of every workload live in generalsparse_amd/autotune.py (CANDIDATES,
# WORKLOAD_CLASS, shape_candidates): the product's search and this bench search the same space.


def kernel_label(info):
    """the device kernel gs_spmm launches (gs_plan_info.device_kernel)"""
    return info.get("device_kernel") or info["kernel_name"]


def algorithmic_bytes(M, K, N, nnz, e, s_idx):
    # each A element once, B read once, C written once
    return nnz * (e + s_idx) + (M + 1) * 4 + K * N * e + M * N * e


def algorithmic_bytes_24(M, K, N, nnz, e):
    # SURVEY.md §8d, 2:4 layout on C3: values + 2-bit positions, B once, C once
    return nnz * e + nnz // 4 + K * N * e + M * N * e


def mark(torch):
    """GS_BENCH_MARK=1: one tiny fill kernel on the current stream, launched right before the
    first and right after the last timed launch, so that scripts/timed_stats.py can keep only
    the timed region's dispatches of a rocprofv3 kernel trace (the plan search's launches of
    the same kernels are left out)"""
    if os.environ.get("GS_BENCH_MARK") == "1":
        torch.cuda._sleep(64)  # a kernel of its own name (spin), launched nowhere else


def time_plan(plan, Bs, Cs, N, steps, warmup, torch, dist=None):
    """returns (host wall seconds for `steps` launches, seconds by HIP events on the launch
    stream over the same `steps` launches), each the max over ranks.  The event time is the
    reference's own measure (GpuTimer around the launches, baseline/base_cusparse/spmm.cu:137-154);
    the wall time adds the host enqueue and the final synchronisation."""
    stream = torch.cuda.current_stream()
    rot = plan.rotation(Bs, Cs)  # operands checked and packed outside the timed region
    rot.run(warmup, 0)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    mark(torch)
    t0 = time.perf_counter()
    e0.record(stream)
    # the rotation continues after the warm-up steps' copies (a timed step never reuses one
    # that a warm-up step left in the Infinity Cache)
    rot.run(steps, warmup)
    e1.record(stream)
    mark(torch)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    wall = t1 - t0
    ev_s = e0.elapsed_time(e1) * 1e-3
    return max_over_ranks(wall, dist, torch), max_over_ranks(ev_s, dist, torch)


def time_plan_combined(plan, Bs, Cs, N, steps, warmup, torch, dist, shards, rank):
    """nnz-exact shards: every step is the local SpMM plus the boundary exchange
    (shard.combine_boundaries: one all-reduce of world x N fp32 over RCCL)"""
    from generalsparse_amd import shard as sd
    reps = len(Bs)

    def one(i):
        plan.spmm(Bs[i % reps], C=Cs[i % reps], replica=i % plan.info()["replicas"])
        sd.combine_boundaries(Cs[i % reps], shards, rank, dist, torch)

    for i in range(warmup):
        one(i)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for i in range(steps):
        one(i)
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dist.barrier()
    return max_over_ranks(wall, dist, torch), max_over_ranks(e0.elapsed_time(e1) * 1e-3, dist, torch)


def max_over_ranks(x, dist, torch):
    """the job's time = the slowest rank's (RCCL on GPU ranks, gloo on CPU ranks)"""
    if dist is None:
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def shard_seed(rank):
    """row-sharded batch: rank r owns its own matrix (seed 13 + r), no exchange"""
    return 13 + rank


def whole_job_gflops(world, flops_per_step, steps, wall_s):
    """value = work of all ranks / the max-over-ranks time (weak scaling)"""
    return world * flops_per_step * steps / wall_s / 1e9


def rocsparse_baseline(M, K, N, row, col, val, copies, dtype, reps=100, warmup=300):
    """best rocSPARSE CSR SpMM algorithm for dtype (1: fp16 A and B, fp32 C and compute
    -- rocSPARSE's documented mixed precision; 0: fp32); None if every algorithm fails.
    300 untimed launches per algorithm before its timed ones (round 6; was 10): the GPU leaves
    the idle clock of the host-side setup before either side is timed (DESIGN.md §4 protocol)"""
    lib = ctypes.CDLL(os.path.join(ROOT, "generalsparse_amd", "librocsparse_cmp.so"))
    lib.rs_last_error.restype = ctypes.c_char_p
    rp = np.zeros(M + 1, np.int64)
    np.add.at(rp, row.astype(np.int64) + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    c32 = col.astype(np.int32)
    v = val.astype(np.float32)
    best = None
    for alg, name in ((0, "default"), (1, "csr"), (4, "csr_row_split"), (5, "csr_nnz_split")):
        ms = ctypes.c_double()
        rc = lib.rs_spmm_bench(M, K, len(v), rp.ctypes.data_as(ctypes.c_void_p), c32.ctypes.data_as(ctypes.c_void_p),
                               v.ctypes.data_as(ctypes.c_void_p), N, dtype, alg, warmup, reps, copies,
                               ctypes.byref(ms), None)
        if rc != 0:
            continue
        gf = 2.0 * len(v) * N / (ms.value * 1e-3) / 1e9
        if best is None or gf > best["gflops"]:
            best = {"gflops": round(gf, 1), "ms": round(ms.value, 5), "alg": name}
    return best


def cpu_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline(M, K, N, row, col, val, min_s=10.0, row_share=1):
    """the oracle's restatement of the reference's host path (checker code, timed
    here only as the CPU baseline): plan transform once + host SpMM repeated, single
    thread as the reference runs it; plus the build's all-cores OpenMP variant of the
    same SpMM (not the reference's).  row_share > 1 times the first M/row_share rows
    only (a bounded sample).  Hot cache: the same A and B every repetition."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as ofi
    what = "full matrix"
    if row_share > 1:
        Ms = M // row_share
        keep = row < Ms
        row, col, val, M = row[keep], col[keep], val[keep], Ms
        what = f"first {Ms} rows (1/{row_share} of the matrix)"
    t_tr, _ = ofi.time_cpu_path(M, K, row, col, val, N)
    t_spmm, reps = ofi.time_spmm_repeated(M, K, row, col, val, N, min_s)
    gf = 2.0 * len(row) * N * reps / t_spmm / 1e9
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    t_mt, reps_mt = ofi.time_spmm_repeated_mt(M, K, row, col, val, N, min_s / 2, threads)
    gf_mt = 2.0 * len(row) * N * reps_mt / t_mt / 1e9
    model, nproc = cpu_info()
    return {"value": round(gf, 3), "unit": "GFLOP/s", "cores": 1, "kind": "port",
            "sample": f"{what}: spmm_reference_host restated (fp32) x{reps} in {t_spmm:.1f} s, "
                      f"single thread; plan transform (thread_total) once {t_tr:.2f} s; hot cache",
            "transform_s": round(t_tr, 3), "spmm_s_per_rep": round(t_spmm / reps, 4),
            "cpu_model": model, "nproc": nproc,
            "multi_thread": {"value": round(gf_mt, 3), "unit": "GFLOP/s", "threads": threads,
                             "label": f"{threads} threads of nproc {nproc} (OMP_NUM_THREADS: the one-GPU box's CPU "
                                      f"share), not all cores",
                             "kind": "the build's OpenMP variant (the reference's host path is single-threaded)",
                             "sample": f"{what} x{reps_mt} in {t_mt:.1f} s"}}


def run_c5(args, torch, gsa, ds, rank, world, local, dev, dist):
    """BASELINE.json configs[4]: the OPT-30B batch split over the ranks by LPT on nnz
    (generalsparse_amd/batch.py); each rank runs its share of SpMMs per step, no
    exchange.  One distinct seeded matrix per shape per rank; every matrix instance of
    the batch streams its own HBM copy of A (a plan replica)."""
    from generalsparse_amd import batch as bt
    N = args.N
    batch, owner, load = bt.c5_assignment(args.layers, world)
    seq = bt.rank_sequence(batch, owner, rank)
    t0 = time.perf_counter()
    # per-shape plan choice (this rank's shapes, its own matrices), then the batch's plans
    choice, per_shape = search_shapes(args, torch, gsa, ds, rank, local, dev, sorted({k for (_, _, k, _) in seq}),
                                      bt.C5_SPARSITY, rocsparse=False)
    plans, launches, _ = bt.build_rank_batch(seq, rank, N, gsa, ds, torch, dev, local, choice=choice)
    t_setup = time.perf_counter() - t0
    step, streams = batch_step(launches, N, torch, args.streams, group=bool(args.group))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall, ev_s = timed_batch(step, streams, args.steps, torch, marked=True)
    wall = max_over_ranks(wall, dist, torch)
    ev_s = max_over_ranks(ev_s, dist, torch)
    if dist is not None:
        dist.barrier()
    total_nnz = sum(bt.nnz_of_shape(b[2]) for b in batch)
    flops = 2.0 * total_nnz * N
    value = flops * args.steps / ev_s / 1e9
    e = 2
    alg = sum(bt.nnz_of_shape(k) * (e + 2) + (bt.C5_SHAPES[k][0] + 1) * 4 + bt.C5_SHAPES[k][1] * N * e +
              bt.C5_SHAPES[k][0] * N * e for (_, _, k) in batch)
    ms = ev_s / args.steps * 1e3
    # HBM bytes per step from the PMC passes of scripts/gpu_traffic_c5.sh (per GPU: the LPT
    # split is balanced on nnz); only for the full 48-layer batch it was scaled to
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic_c5.json")
    kinds = {kernel_label(p.info()) for p in plans.values()}
    if os.path.exists(tf) and args.layers == 48:
        try:
            tj = json.load(open(tf))
            if "+".join(sorted(kinds)) == tj.get("kernel"):  # measured on the same kernels
                traffic = int(tj["hbm_bytes_per_step"] / world)
        except Exception:
            traffic = None
    out = {
        "metric": "SpMM GFLOP/s, OPT-30B 80%-pruned weight batch fp16 N=32 (configs[4])",
        "value": round(value, 1), "unit": "GFLOP/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "timing": "HIP events around the K timed steps (all streams joined), max over ranks",
        "wall_ms_per_step": round(wall / args.steps * 1e3, 4),
        "dtype": "f16 (fp32 accumulate)",
        "data": "synthetic (one seeded magnitude-pruned Gaussian per shape per rank; each batch instance streams "
                "its own HBM copy of A)",
        "config": {"workload": f"OPT-30B weight batch: {args.layers} layers x (4 x 7168^2, 28672x7168, 7168x28672), "
                               f"80% unstructured, fp16, N={N}", "matrices": len(batch), "nnz": total_nnz,
                   "plan": {k: per_shape[k]["plan"] for k in plans},
                   "kernel": {k: kernel_label(plans[k].info()) for k in plans},
                   "parallelism": f"LPT batch split x{world} (max rank nnz share {max(load) / total_nnz:.4f})",
                   "streams": args.streams, "grouped_launches": bool(args.group)},
        "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9 / world, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / world / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "algorithmic_bytes_per_step": alg, "note": "per GPU, whole step"},
        "setup_s": round(t_setup, 1),
        "per_shape": {k: {x: v[x] for x in ("plan", "kernel", "kernel_us", "hbm_frac")} for k, v in per_shape.items()},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    for p in plans.values():
        p.free()


def timed_batch(step, streams, steps, torch, marked=False):
    """`steps` calls of a batch step over its streams; returns (host wall s, HIP-event s).
    The events sit on the first stream; the other streams wait for the start event and the
    first stream waits for their last launches before the stop event."""
    cur = streams[0]
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if marked:
        mark(torch)
    t0 = time.perf_counter()
    e0.record(cur)
    for s in streams[1:]:
        s.wait_event(e0)
    for _ in range(steps):
        step()
    for s in streams[1:]:
        cur.wait_event(s.record_event())
    e1.record(cur)
    if marked:
        mark(torch)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, e0.elapsed_time(e1) * 1e-3


def batch_step(launches, N, torch, n_streams, group=False):
    """one pass over a batch of independent SpMMs.  group: the batch through gs_spmm_batch
    (consecutive K-split entries of one instantiation are one grouped launch; entries sorted
    largest matrix first, same shapes together, then dealt over the streams), every launch with its own C.  Otherwise launch i on stream i % n_streams (the current stream first), so
    one launch's tail overlaps the next one's start; with more than one stream every launch
    writes its own C.  Returns (step, streams)."""
    import generalsparse_amd as gsa
    cur = torch.cuda.current_stream()
    streams = [cur] + [torch.cuda.Stream() for _ in range(max(1, n_streams) - 1)]
    if group:
        # sorted by shape, then dealt over the streams: each stream's share is one batch of
        # long same-shape runs, and the streams' grouped launches overlap each other's tails
        # largest matrices first (their workgroups run longest: a grouped launch dispatches its
        # entries in order, so the short ones fill the tail), same shapes together
        ents = [(p, r, b, torch.empty_like(c), k)
                for (p, r, b, c, k) in sorted(launches, key=lambda x: (-x[3].shape[0] * x[2].shape[0], x[4]))]
        bats = [(gsa.Batch([(p, r, b, c) for (p, r, b, c, _) in ents[i::len(streams)]], N), st.cuda_stream)
                for i, st in enumerate(streams) if ents[i::len(streams)]]

        def gstep():
            for bat, s in bats:
                bat.run(s)

        gstep.keep = ents  # the C buffers live as long as the step
        gstep.launches = lambda: [n for bat, _ in bats for n in bat.launches()]  # entries per launch
        return gstep, streams
    raw = []
    for i, (p, r, b, c, _) in enumerate(launches):
        if n_streams > 1:
            c = torch.empty_like(c)
        raw.append((p, r, b.data_ptr(), c.data_ptr(), streams[i % len(streams)].cuda_stream, c))

    def step():
        for plan, r, b, c, s, _ in raw:
            plan.spmm_raw(b, c, N, r, s)

    return step, streams


def search_shapes(args, torch, gsa, ds, rank, local, dev, shapes, sp, rocsparse=True):
    """per shape: every generalsparse_amd.batch.shape_candidates plan timed by events with
    rotated replicas (the plan search obtain_result.py does), the best kept as the shape's
    choice; rocSPARSE 7.2 CSR SpMM (fp16 A/B, fp32 C) on the same matrix beside it"""
    from generalsparse_amd import batch as bt
    N, e = args.N, 2
    choice, per_shape = {}, {}
    for k in shapes:
        m, n = bt.C5_SHAPES[k]
        row, col, val = ds.pruned_weight(m, n, sp, bt.shape_seed(rank, k))
        nnz = len(row)
        flops = 2.0 * nnz * N
        alg = algorithmic_bytes(m, n, N, nnz, e, 2)
        best, variants = None, {}
        for cand in bt.shape_candidates(k):
            key = "%s(%d,%d)%s" % (cand[0], cand[1], cand[2], "".join(f" {a}={b}" for a, b in cand[3].items()))
            try:
                plan = bt.build_plan(gsa, m, n, row, col, val, N, cand, local)
            except gsa.GsError as ex:
                variants[key] = {"error": str(ex)}
                continue
            except Exception as ex:  # noqa: BLE001 -- recorded with the shape, never a silent skip
                variants[key] = {"error": f"{type(ex).__name__}: {ex}"}
                continue
            info = plan.info()
            reps = replicas_for(info, n, N, e, args.rotation_mb)
            for _ in range(reps - 1):
                plan.add_replica()
            Bs = [torch.randn((n, N), device=dev, dtype=torch.float16) for _ in range(reps)]
            Cs = [torch.empty((m, N), device=dev, dtype=torch.float16) for _ in range(reps)]
            ms = event_ms(plan, Bs, Cs, args.search_reps, torch)
            variants[key] = {"kernel": kernel_label(info), "kernel_us": round(ms * 1e3, 2)}
            if best is None or ms < best[0]:
                best = (ms, cand, key, kernel_label(info), reps)
            plan.free()
            del Bs, Cs
            torch.cuda.empty_cache()
        if best is None:  # every candidate of the shape failed: report them, do not crash
            print(json.dumps({"error": f"no plan runs for shape {k}", "shape": k, "variants": variants}), flush=True)
            raise SystemExit(1)
        ms, cand, key, kern, reps = best
        choice[k] = cand
        rs = rocsparse_baseline(m, n, N, row, col, val, min(reps, 20), dtype=1) if rocsparse else None
        per_shape[k] = {"M": m, "K": n, "nnz": nnz, "plan": key, "kernel": kern, "kernel_us": round(ms * 1e3, 2),
                        "gflops": round(flops / (ms * 1e-3) / 1e9, 1),
                        "hbm_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "variants": variants,
                        "rocsparse_f16": rs,
                        "speedup_vs_rocsparse": round(rs["ms"] / ms, 3) if rs else None}
        del row, col, val
    return choice, per_shape


# the headline layer's plan when no search runs (the default bench line's north_star object):
# block_total(112,1) on all six slots -- the r04 layer search's pick (profiles/r04y_c5h_bench.json:
# attn, fc1 and fc2 on 112-row k_mfma_ks blocks, the layer ONE grouped launch)
HEADLINE_CHOICE = ("block_total", 112, 1, {})
NORTH_STAR_TARGET = {"speedup_vs_rocsparse": 1.5, "hbm_frac": 0.5}
# the copy rate MI355X_MICROARCH.md measures with a tuned kernel (GB/s): the practical HBM ceiling
GUIDE_COPY_GBS = 6290.0


def layer_consts(N, sp):
    """(nnz, flops, algorithmic bytes) of one OPT-30B layer step (six SpMMs)"""
    from generalsparse_amd import batch as bt
    nnz_l = sum(bt.nnz_of_shape(k, sp) for k in bt.C5_SLOTS)
    alg_l = sum(algorithmic_bytes(*bt.C5_SHAPES[k], N, bt.nnz_of_shape(k, sp), 2, 2) for k in bt.C5_SLOTS)
    return nnz_l, 2.0 * nnz_l * N, alg_l


def layer_traffic(N, sp, plans_by_shape):
    """L2->fabric bytes of the layer step from the PMC passes of the headline candidates
    (profiles/traffic_c5h.json, per (shape, plan)); None unless every slot's plan was measured"""
    from generalsparse_amd import batch as bt
    tf = os.path.join(ROOT, "profiles", "traffic_c5h.json")
    if not os.path.exists(tf):
        return None, {}
    try:
        tj = json.load(open(tf))
        if tj["N"] != N or abs(tj["sparsity"] - sp) > 1e-9:
            return None, {}
        pl = tj["per_launch"]
        per = {k: pl.get(k, {}).get(plans_by_shape[k], {}).get("hbm_bytes") for k in plans_by_shape}
        if all(per.get(k) for k in bt.C5_SLOTS):
            return sum(per[k] for k in bt.C5_SLOTS), per
        return None, per
    except Exception:
        return None, {}


def cand_key(c):
    from generalsparse_amd.autotune import cand_key as ck
    return ck(c)


def headline_layer(args, torch, gsa, ds, rank, local, dev, choice, steps, warmup, per_shape=None, rs_per_shape=None,
                   settle_ms=0.0):
    """The north_star headline: one OPT-30B decoder layer's six pruned weights
    (q, k, v, out 7168^2; fc1 28672x7168; fc2 7168x28672) at `args.sparsity`, fp16, N=32, one
    GPU, with the per-shape plans of `choice`.  The timed step = the layer's six SpMMs, one plan
    replica per instance (the layer's A is ~750 MB, past the 256 MB Infinity Cache), through
    gs_spmm_batch (grouped k_mfma_ks launches) when args.group.  With `per_shape` (the c5h
    search's results) and grouped launches, attn's K-split alternatives within 15% are also
    timed as whole layers and the fastest layer kept.  Returns (line dict, plans, step)."""
    from generalsparse_amd import batch as bt
    N, sp = args.N, args.sparsity
    seq = [(0, s, bt.C5_SLOTS[s], bt.C5_SLOTS[:s].count(bt.C5_SLOTS[s])) for s in range(len(bt.C5_SLOTS))]

    def build_layer(ch):
        plans, launches, coo = bt.build_rank_batch(seq, rank, N, gsa, ds, torch, dev, local, sparsity=sp, choice=ch,
                                                   keep_coo=rs_per_shape is None and not args.no_rocsparse)
        step, streams = batch_step(launches, N, torch, args.streams, group=bool(args.group))
        return plans, step, streams, coo

    plans, step, streams, coo = build_layer(choice)
    layer_search = None
    if args.group and per_shape is not None:
        ks = sorted((v["kernel_us"], key) for key, v in per_shape["attn"]["variants"].items()
                    if v.get("kernel") == "k_mfma_ks")
        cands = {cand_key(c): c for c in bt.shape_candidates("attn")}
        alts = [key for us, key in ks if us <= 1.15 * ks[0][0] and key != per_shape["attn"]["plan"]] if ks else []
        if alts:
            best_ms = layer_ms(step, streams, torch)
            layer_search = {"per_shape_best": {"attn": per_shape["attn"]["plan"], "layer_ms": round(best_ms, 5)},
                            "attn_alternatives": {}, "kept": per_shape["attn"]["plan"]}
            for alt_key in alts:
                plans2, step2, streams2, _ = build_layer(dict(choice, attn=cands[alt_key]))
                t_b = layer_ms(step2, streams2, torch)
                layer_search["attn_alternatives"][alt_key] = round(t_b, 5)
                if t_b < best_ms:
                    for p in plans.values():
                        p.free()
                    plans, step, streams, best_ms = plans2, step2, streams2, t_b
                    layer_search["kept"] = alt_key
                else:
                    for p in plans2.values():
                        p.free()
                del step2
            if layer_search["kept"] != per_shape["attn"]["plan"]:
                e = 2
                k2 = layer_search["kept"]
                ps = per_shape["attn"]
                ps["plan_alone_best"] = ps["plan"]
                ps["plan"], ps["kernel"], ps["kernel_us"] = k2, ps["variants"][k2]["kernel"], ps["variants"][k2]["kernel_us"]
                ps["gflops"] = round(2.0 * ps["nnz"] * N / (ps["kernel_us"] * 1e-6) / 1e9, 1)
                ps["hbm_frac"] = round(algorithmic_bytes(ps["M"], ps["K"], N, ps["nnz"], e, 2)
                                       / (ps["kernel_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    launches_per_step = step.launches() if hasattr(step, "launches") else None
    # settle_ms: untimed layer steps until that much time has passed (the layer's plans are built
    # on the host while the GPU idles; an idle MI355X lowers its clock, and the first tens of ms of
    # work after it run slower: 20 timed steps after 10 read 0.45 of HBM, 200 after 20 0.54,
    # profiles/r05x_steps.txt), then the warm-up steps and the timed ones
    n_settle = 0
    if settle_ms > 0:
        t_s = time.perf_counter()
        while (time.perf_counter() - t_s) * 1e3 < settle_ms:
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            n_settle += 10
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    wall, ev_s = timed_batch(step, streams, steps, torch, marked=True)
    ms_step = ev_s / steps * 1e3
    nnz_l, flops_l, alg_l = layer_consts(N, sp)
    plan_of = {k: (per_shape[k]["plan"] if per_shape else cand_key(choice[k])) for k in bt.C5_SHAPES}
    traffic, traffic_per = layer_traffic(N, sp, plan_of)
    if rs_per_shape is None and not args.no_rocsparse:
        rs_per_shape = {}
        for k, (m, n) in bt.C5_SHAPES.items():
            row, col, val = coo[k]
            copies = max(2, int(math.ceil(args.rotation_mb * 1e6 / (len(row) * 6 + n * N * 2))))
            rs_per_shape[k] = rocsparse_baseline(m, n, N, row, col, val, min(copies, 20), dtype=1)
    rs_l = None
    if rs_per_shape and all(rs_per_shape.get(k) for k in bt.C5_SHAPES):
        rs_l = sum(rs_per_shape[k]["ms"] for k in bt.C5_SLOTS)
    frac = alg_l / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS
    line = {
        "metric": "SpMM GFLOP/s + achieved HBM GB/s vs rocSPARSE, OPT-30B %d%%-pruned layer fp16 N=32 (north_star headline)"
                  % round(sp * 100),
        "value": round(flops_l * steps / ev_s / 1e9, 1), "unit": "GFLOP/s", "steps": steps, "warmup": warmup,
        "settle_steps": n_settle, "settle_ms": settle_ms,
        "ms_per_step": round(ms_step, 5), "higher_is_better": True,
        "timing": "HIP events around the K timed steps (all streams joined)",
        "wall_ms_per_step": round(wall / steps * 1e3, 5),
        "dtype": "f16 (fp32 accumulate)",
        "data": "synthetic (one seeded magnitude-pruned Gaussian per shape; each layer instance streams its own HBM "
                "copy of A); OPT-30B weights are not available offline",
        "config": {"workload": f"OPT-30B decoder layer: 4 x 7168^2, 28672x7168, 7168x28672, {round(sp * 100)}% "
                               f"unstructured, fp16, N={N}", "nnz": nnz_l, "plan": plan_of,
                   "kernel": {k: kernel_label(plans[k].info()) for k in plans},
                   "launches_per_step": launches_per_step, "streams": args.streams,
                   "grouped_launches": bool(args.group)},
        "roofline": {"bound": "hbm", "achieved": round(alg_l / (ms_step * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(frac, 4), "traffic": traffic, "algorithmic_bytes_per_step": alg_l,
                     "note": "whole layer step (HIP events); traffic = the PMC bytes of the same (shape, plan) "
                             "launches, profiles/traffic_c5h.json"},
        "speedup_vs_rocsparse": round(rs_l / ms_step, 3) if rs_l else None,
        "rocsparse_layer_ms": round(rs_l, 4) if rs_l else None,
        "rocsparse_per_shape": rs_per_shape,
        "layer_search": layer_search,
    }
    line["target"] = dict(NORTH_STAR_TARGET)
    line["met"] = bool(rs_l and rs_l / ms_step >= NORTH_STAR_TARGET["speedup_vs_rocsparse"]
                       and frac >= NORTH_STAR_TARGET["hbm_frac"])
    if traffic_per:
        line["traffic_per_launch"] = traffic_per
    return line, plans


def run_c5h(args, torch, gsa, ds, rank, world, local, dev, dist):
    """north_star headline as its own line: the per-shape plan search over
    generalsparse_amd.batch.shape_candidates (event time with rotated replicas, rocSPARSE 7.2
    CSR SpMM fp16 A/B fp32 C on the same matrix), the layer-level attn choice, then the timed
    layer (headline_layer)."""
    from generalsparse_amd import batch as bt
    N, sp = args.N, args.sparsity
    choice, per_shape = search_shapes(args, torch, gsa, ds, rank, local, dev, list(bt.C5_SHAPES), sp,
                                      rocsparse=not args.no_rocsparse)
    rs = {k: per_shape[k]["rocsparse_f16"] for k in per_shape} if not args.no_rocsparse else {}
    out, plans = headline_layer(args, torch, gsa, ds, rank, local, dev, choice, args.steps, args.warmup,
                                per_shape=per_shape, rs_per_shape=rs, settle_ms=200.0)
    nnz_l, flops_l, alg_l = layer_consts(N, sp)
    # the layer's kernels one at a time (each shape's search time = its own launch alone)
    serial_ms = sum(per_shape[k]["kernel_us"] for k in bt.C5_SLOTS) * 1e-3
    out["serial_kernels"] = {"ms": round(serial_ms, 5), "gflops": round(flops_l / (serial_ms * 1e-3) / 1e9, 1),
                             "hbm_frac": round(alg_l / (serial_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "note": "sum of the six launches timed alone (per_shape kernel_us)"}
    for k in per_shape:
        per_shape[k]["traffic"] = out.get("traffic_per_launch", {}).get(k)
    out.update({"n_gpus": world, "scaling": "weak", "vs_baseline": None, "per_shape": per_shape})
    out["config"]["parallelism"] = "one GPU"
    if rank == 0:
        print(json.dumps(out), flush=True)
    for p in plans.values():
        p.free()


def layer_ms(step, streams, torch, warm=10, reps=30):
    """event time (ms) of one layer step, all streams joined (the c5h layer-level choice)"""
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    _, ev_s = timed_batch(step, streams, reps, torch)
    return ev_s / reps * 1e3


def replicas_for(info, K, N, e, rotation_mb):
    """independent copies of A and B so the rotation set covers rotation_mb of the bytes
    the launched kernel actually reads (the matrix-core layouts, not a deferred CSR)"""
    read_A = info["tile_bytes"] if info["lds_stage"] in (2, 3) and info["tile_bytes"] else info["device_bytes_A"]
    return max(2, int(math.ceil(rotation_mb * 1e6 / (read_A + K * N * e))))


def stream_copy_gbs(torch, dev, mib=2048, reps=10):
    """STREAM-copy bandwidth of this GPU (SURVEY 8d's measured denominator): a torch copy of
    `mib` MiB of fp32, read + written bytes over the HIP-event time of `reps` copies"""
    n = mib * (1 << 20) // 4
    a = torch.empty(n, dtype=torch.float32, device=dev).uniform_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2.0 * n * 4 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return round(gbs, 1)


def settle_gpu(plan, Bs, Cs, torch, ms):
    """untimed rotated launches of `plan` until `ms` milliseconds of wall time have passed: the
    GPU lowers its clock while the host builds a plan, and the first tens of ms of work after
    such a gap run slower (DESIGN.md §4 protocol notes)"""
    rot = plan.rotation(Bs, Cs)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        rot.run(20, 0)
        torch.cuda.synchronize()


def event_ms(plan, Bs, Cs, reps, torch, warm=20, rotate=True):
    """average kernel time (ms) of `reps` launches from HIP events on the launch stream"""
    stream = torch.cuda.current_stream()
    rot = plan.rotation(Bs, Cs)  # operands checked once, outside the timed launches
    b0, c0, N, s = Bs[0].data_ptr(), Cs[0].data_ptr(), Bs[0].shape[1], stream.cuda_stream
    if rotate:
        rot.run(warm, 0)
    else:
        for _ in range(warm):
            plan.spmm_raw(b0, c0, N, 0, s)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    if rotate:
        rot.run(reps, 0)
    else:
        for _ in range(reps):
            plan.spmm_raw(b0, c0, N, 0, s)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def build_plan(gsa, M, K, row, col, val, cand, N, dt, local, rotation_mb, e, tdt, dev, torch):
    """a candidate's plan with its replicas and B / C buffers; cand = (pipeline, p0, p1[, config
    overrides held while the plan is compiled and uploaded])"""
    from generalsparse_amd.autotune import build_candidate
    t0 = time.perf_counter()
    plan = build_candidate(M, K, row, col, val, cand, N, dt, local)
    t_plan = time.perf_counter() - t0  # transforms + compile + upload
    info = plan.info()
    reps = replicas_for(info, K, N, e, rotation_mb)
    for _ in range(reps - 1):
        plan.add_replica()
    Bs = [torch.randn((K, N), device=dev, dtype=tdt) for _ in range(reps)]
    Cs = [torch.empty((M, N), device=dev, dtype=tdt) for _ in range(reps)]
    return plan, Bs, Cs, reps, t_plan


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: every rank on cuda:0, the barrier and the
    # max-over-ranks on gloo (RCCL takes one rank per device).  Timings are contended: the line
    # is a functional check of the multi-rank path, never a scaling number.
    shared = os.environ.get("GS_BENCH_SHARED_GPU") == "1" and world > 1
    if shared:
        local = 0
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the real world size",
              file=sys.stderr, flush=True)
    resolve_workload(args, world)
    dist = None
    if world > 1:
        import torch.distributed as td
        torch.cuda.set_device(local)
        if shared:
            td.init_process_group("gloo")
        else:
            td.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        dist = td
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")

    import generalsparse_amd as gsa
    from generalsparse_amd import datasets as ds
    for kv in args.config:
        k, v = kv.split("=", 1)
        gsa.set_config(k, int(v))

    if args.workload == "c5h":
        run_c5h(args, torch, gsa, ds, rank, world, local, dev, dist)
        if dist is not None:
            dist.destroy_process_group()
        return
    if args.workload == "c5":
        run_c5(args, torch, gsa, ds, rank, world, local, dev, dist)
        if dist is not None:
            dist.destroy_process_group()
        return
    from generalsparse_amd import autotune as at
    M, K, N = args.M, args.K, args.N
    wl = WORKLOADS[args.workload]
    dt = wl["dtype"]
    tdt = torch.float16 if dt == "f16" else torch.float32
    e, s_idx = (2 if dt == "f16" else 4), (2 if K <= 65536 else 4)
    shards = None
    if args.workload == "c1":
        row, col, val = ds.random_rows(M, K, 1790490 / 47894, 18)
        nnz = len(row)
        alg_bytes = algorithmic_bytes(M, K, N, nnz, e, s_idx)
        cand_list = at.CANDIDATES[at.WORKLOAD_CLASS["c1"]]
    elif args.workload in ("c4", "c4o"):
        one = args.shard != "batch"
        if args.workload == "c4o":  # 234M nonzeros: drawn on the GPU (numpy takes minutes)
            row, col, val = ds.rmat_torch(M, wl["nnz"], wl["seed"] + (0 if one else rank), dev, symmetric=True)
            cand_list = at.CANDIDATES[at.WORKLOAD_CLASS["c4o"]]
        else:
            row, col, val = ds.rmat(M, wl["nnz"], wl["seed"] + (0 if one else rank), symmetric=wl["symmetric"])
            cand_list = at.CANDIDATES[at.WORKLOAD_CLASS["c4"]]
        nnz = len(row)
        alg_bytes = algorithmic_bytes(M, K, N, nnz, e, s_idx)
        if one:  # one matrix over the ranks: this rank's rows / nonzeros
            from generalsparse_amd import shard as sd
            full_flops = 2.0 * nnz * N
            shards = (sd.nnz_exact_shards if args.shard == "nnz" else sd.balanced_row_shards)(row, M, world)
            M, row, col, val = sd.local_coo(row, col, val, shards[rank])
    elif args.workload == "c3":
        row, col, val = ds.two_four(M, K, 30 + rank)
        nnz = len(row)
        alg_bytes = algorithmic_bytes_24(M, K, N, nnz, e)
        cand_list = at.CANDIDATES[at.WORKLOAD_CLASS["c3"]]
    else:
        row, col, val = ds.pruned_weight(M, K, args.sparsity, shard_seed(rank))
        nnz = len(row)
        alg_bytes = algorithmic_bytes(M, K, N, nnz, e, s_idx)
        cand_list = at.CANDIDATES[at.WORKLOAD_CLASS["c2"]]
    flops = 2.0 * nnz * N

    cands = cand_list if args.pipeline == "auto" else [c for c in cand_list if c[0] == args.pipeline] or \
        [(args.pipeline, 0, 1)]
    if args.p0 is not None:  # one variant (profiling runs)
        cands = [(c[0], args.p0, c[2] if args.p1 is None else args.p1) for c in cands[:1]]
    # plan search (obtain_result.py's best variant): every candidate built, then timed in
    # `--search-rounds` interleaved rounds of search_reps launches each; a candidate's time is
    # its median over the rounds (max over ranks, so every rank keeps the same plan).
    # Interleaving and the median keep candidates within a few percent of each other from
    # flipping the choice with the chip's clock from run to run.
    # (matrices of more than 50M nonzeros -- the com-Orkut stand-in -- are built and timed one
    # candidate at a time, one round, so that only one candidate's host and device copies live)
    variants = {}
    built = []
    one_at_a_time = nnz > 50_000_000
    rounds = 1 if one_at_a_time else max(1, args.search_rounds)
    best = None
    # the candidates that lost are freed after the timed region (one at a time: at once), so the
    # device does not sit idle in hipFree between the search's last launches and the timed steps
    # (an idle GPU lowers its clock: the first steps after a gap run slower)
    losers = []

    def drop(p_):
        if one_at_a_time:
            p_.free()
        else:
            losers.append(p_)

    def settle(b):
        nonlocal best
        plan_, Bs_, Cs_, reps_, cand_, key_, info_, t_plan_, times_ = b
        ms_ = float(np.median(times_))
        variants[key_] = {"kernel_ms": round(ms_, 5), "rounds_ms": [round(t, 5) for t in times_],
                          "gflops_per_gpu": round(flops / (ms_ * 1e-3) / 1e9, 1),
                          "kernel": kernel_label(info_), "replicas": reps_, "plan_s": round(t_plan_, 2)}
        if best is None or ms_ < best[0]:
            if best is not None:
                drop(best[1])
            best = (ms_, plan_, Bs_, Cs_, reps_, cand_, key_, info_)
        else:
            drop(plan_)

    for cand in cands:
        key = cand_key(cand)
        try:
            plan, Bs, Cs, reps, t_plan = build_plan(gsa, M, K, row, col, val, cand, N, dt, local, args.rotation_mb, e,
                                                    tdt, dev, torch)
        except gsa.GsError as ex:  # e.g. the balanced splitter on trailing empty rows
            variants[key] = {"error": str(ex)}
            continue
        b = [plan, Bs, Cs, reps, cand, key, plan.info(), t_plan, []]
        if one_at_a_time:
            b[8].append(max_over_ranks(event_ms(plan, Bs, Cs, args.search_reps, torch), dist, torch))
            settle(b)
            del b, Bs, Cs
            torch.cuda.empty_cache()
        else:
            built.append(b)
    for _ in range(rounds if built else 0):
        for b in built:
            b[8].append(max_over_ranks(event_ms(b[0], b[1], b[2], args.search_reps, torch), dist, torch))
    for b in built:
        settle(b)
    del built
    if best is None:
        print(json.dumps({"metric": wl["metric"], "error": "no candidate plan runs", "variants": variants}), flush=True)
        raise SystemExit(1)
    _, plan, Bs, Cs, reps, best_cand, key, info = best
    # the measurement: W untimed warm-up steps, exactly K timed steps
    if shards is not None and args.shard == "nnz" and dist is not None:
        wall, ev_s = time_plan_combined(plan, Bs, Cs, N, args.steps, args.warmup, torch, dist, shards, rank)
    else:
        wall, ev_s = time_plan(plan, Bs, Cs, N, args.steps, args.warmup, torch, dist)
    hot_ms = event_ms(plan, Bs, Cs, 100, torch, rotate=False)
    for p_ in losers:
        p_.free()
    losers.clear()
    torch.cuda.empty_cache()
    copy_gbs = stream_copy_gbs(torch, dev)
    # value and ms_per_step from the HIP events around the K timed steps (max over ranks);
    # the host wall time of the same region is reported beside them
    ev_ms = ev_s / args.steps * 1e3
    ms_per_step = ev_ms
    value = whole_job_gflops(world, flops, args.steps, ev_s)
    wall_value = whole_job_gflops(world, flops, args.steps, wall)
    if shards is not None:  # strong scaling: the job is one matrix
        value = full_flops * args.steps / ev_s / 1e9
        wall_value = full_flops * args.steps / wall / 1e9
    achieved = alg_bytes / (ev_ms * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    if os.path.exists(tf):
        try:
            tj = json.load(open(tf))
            if tj.get("kernel") in (None, kernel_label(info)) and tj.get("plan") in (None, key):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # matrix-core utilisation of the same kernel from its SQ / GRBM PMC pass (scripts/mfma_util.py)
    mfma = None
    mf = os.path.join(ROOT, "profiles", f"mfma_{args.workload}.json")
    if os.path.exists(mf) and kernel_label(info).startswith(("k_mfma", "k_nm")):
        try:
            mj = json.load(open(mf))
            if mj.get("kernel") == kernel_label(info) and mj.get("plan") in (None, key):
                mfma = {k: mj[k] for k in ("mfma_util", "formula", "mfma_util_at_clock_est", "clock_ghz_est", "analytic", "kernel_ns_median")
                        if k in mj}
                mfma["source"] = os.path.relpath(mf, ROOT)
        except Exception:
            mfma = None
    out = {
        "metric": wl["metric"],
        "value": round(value, 1), "unit": "GFLOP/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
        "timing": "HIP events on the launch stream around the K timed steps, max over ranks",
        "wall_ms_per_step": round(wall / args.steps * 1e3, 5), "wall_value": round(wall_value, 1),
        "scaling": "weak" if shards is None else "strong", "vs_baseline": None,
        "dtype": "f16 (fp32 accumulate)" if dt == "f16" else "f32", "data": wl["data"],
        "config": {"workload": wl["workload"].format(M=M, K=K, N=N),
                   "M": M, "K": K, "N": N, "nnz": nnz, "plan": key, "kernel": kernel_label(info),
                   "replicas_rotated": reps, "rotated_read_bytes_per_replica": info["tile_bytes"] or info["device_bytes_A"],
                   "parallelism": f"row-sharded batch x{world}" if shards is None else
                   f"one matrix, {args.shard} shards x{world}" + (" + boundary all-reduce" if args.shard == "nnz" else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": alg_bytes, "kernel_ms": round(ev_ms, 5),
                     "hot_cache_kernel_ms": round(hot_ms, 5),
                     "measured_copy_gbs": copy_gbs, "frac_of_measured_copy": round(achieved / copy_gbs, 4),
                     "guide_copy_gbs": GUIDE_COPY_GBS, "frac_of_guide_copy": round(achieved / GUIDE_COPY_GBS, 4),
                     "measured_copy_note": "STREAM copy measured on this GPU after the timed region (SURVEY 8d): "
                                           "torch's copy of 2 GiB fp32, bytes read + written -- not a tuned copy "
                                           "kernel, so it reads below the 6.29 TB/s MI355X_MICROARCH.md measures "
                                           "(guide_copy_gbs); `peak` stays the 8 TB/s datasheet figure",
                     "mfma_util": mfma["mfma_util"] if mfma else None, "mfma": mfma},
        "variants": variants,
    }
    if args.n_sweep and rank == 0:
        out["n_sweep"] = n_sweep(gsa, M, K, row, col, val, cands, args, dt, local, e, tdt, dev, torch, nnz)
    if rank == 0 and not args.no_rocsparse:
        try:
            out.update(rocsparse_compare(gsa, M, K, N, row, col, val, dt, cands, args, local, flops, ev_ms, dev,
                                         torch, min(reps, 20)))
        except Exception as ex:  # comparator problems must not hide the main number
            out["rocsparse"] = {"error": str(ex)}
    if rank == 0 and world == 1 and not args.no_cpu:
        share = {"c3": 8, "c4o": 64}.get(args.workload, 1)
        out["cpu_baseline"] = cpu_baseline(M, K, N, row, col, val, row_share=share)
    plan.free()
    del Bs, Cs
    torch.cuda.empty_cache()
    if args.workload == "c2" and world == 1 and not args.no_north_star and args.N == 32:
        # the north_star target (OPT-30B 70%-pruned weights at N=32, >= 1.5x rocSPARSE and >= 50%
        # of HBM) timed in the same run: one layer, the headline plans, no search
        from generalsparse_amd import batch as bt
        a2 = argparse.Namespace(**vars(args))
        a2.group, a2.streams = 1, 1
        try:
            # the reference's protocol (100 timed launches after 10 warm-ups, baseline/base_cusparse/
            # spmm.cu:136-158) after 200 ms of untimed layer steps (the plans are built while the GPU idles)
            ns, plans = headline_layer(a2, torch, gsa, ds, rank, local, dev, {k: HEADLINE_CHOICE for k in bt.C5_SHAPES},
                                       max(args.steps, 100), max(args.warmup, 10), settle_ms=200.0)
            for p in plans.values():
                p.free()
            ns["roofline"]["measured_copy_gbs"] = copy_gbs
            ns["roofline"]["frac_of_measured_copy"] = round(ns["roofline"]["achieved"] / copy_gbs, 4)
            ns["roofline"]["frac_of_guide_copy"] = round(ns["roofline"]["achieved"] / GUIDE_COPY_GBS, 4)
            out["north_star"] = ns
        except Exception as ex:  # the C2 line must not be lost to a failure of the extra object
            out["north_star"] = {"error": f"{type(ex).__name__}: {ex}"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def n_sweep(gsa, M, K, row, col, val, cands, args, dt, local, e, tdt, dev, torch, nnz):
    """the workload's plan search at other dense widths (N in {8, 32, 128}): per N
    every candidate plan is built for that N and timed (events, rotated replicas); the fastest
    is reported with its kernel and HBM roofline fraction (algorithmic bytes at that N)"""
    out = []
    s_idx = 2 if K <= 65536 else 4
    for n in [int(x) for x in args.n_sweep.split(",") if x]:
        tried, best = {}, None
        for cand in cands:
            key = cand_key(cand)
            try:
                plan, Bs, Cs, reps, _ = build_plan(gsa, M, K, row, col, val, cand, n, dt, local, args.rotation_mb, e,
                                                   tdt, dev, torch)
            except gsa.GsError as ex:
                tried[key] = {"error": str(ex)[:80]}
                continue
            ms = event_ms(plan, Bs, Cs, args.search_reps, torch)
            kern = kernel_label(plan.info())
            tried[key] = {"kernel": kern, "kernel_ms": round(ms, 5)}
            if best is None or ms < best[0]:
                best = (ms, key, kern)
            plan.free()
            del Bs, Cs
            torch.cuda.empty_cache()
        if best is None:
            out.append({"N": n, "error": "no candidate plan runs", "tried": tried})
            continue
        ms, key, kern = best
        alg = (algorithmic_bytes_24(M, K, n, nnz, e) if args.workload == "c3" else
               algorithmic_bytes(M, K, n, nnz, e, s_idx))
        out.append({"N": n, "plan": key, "kernel": kern, "kernel_ms": round(ms, 5),
                    "gflops": round(2.0 * nnz * n / (ms * 1e-3) / 1e9, 1),
                    "hbm_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "tried": tried})
    return out


def rocsparse_compare(gsa, M, K, N, row, col, val, dt, cands, args, local, flops, ev_ms, dev, torch, copies):
    """rocSPARSE CSR SpMM on the same matrix (cold: rotated copies), fp16 inputs against
    ours at fp16 and fp32 against ours at fp32.  Ours at fp32 is the workload's own plan
    search run at fp32 (every candidate built for f32 data, timed with the same rotation rule,
    the fastest kept: the reference's best-variant search per precision, obtain_result.py)."""
    rs32 = rocsparse_baseline(M, K, N, row, col, val, copies, dtype=0)
    res = {"rocsparse": {"f32": rs32}}
    ours = flops / (ev_ms * 1e-3) / 1e9
    if dt == "f32":
        if rs32:
            res["speedup_vs_rocsparse"] = round(ours / rs32["gflops"], 3)
        return res
    rs16 = rocsparse_baseline(M, K, N, row, col, val, copies, dtype=1)
    res["rocsparse"]["f16"] = rs16 if rs16 else "every algorithm failed"
    res["rocsparse"]["f16_note"] = "fp16 A and B, fp32 C and compute (rocsparse_spmm.h mixed precision)"
    if rs16:
        res["speedup_vs_rocsparse"] = round(ours / rs16["gflops"], 3)
    tried, best32 = {}, None
    from generalsparse_amd import autotune as at
    extra = at.F32_EXTRA.get(at.WORKLOAD_CLASS.get(args.workload, ""), []) if args.pipeline == "auto" else []
    for cand in list(cands) + [c for c in extra if c not in cands]:
        if len(cand) > 3:  # config variants of the fp16 matrix-core kernels (KS_NT, NM_NT): no fp32 plan
            continue
        key = cand_key(cand)
        try:
            plan, Bs, Cs, reps, _ = build_plan(gsa, M, K, row, col, val, cand, N, "f32", local, args.rotation_mb, 4,
                                               torch.float32, dev, torch)
        except gsa.GsError as ex:
            tried[key] = {"error": str(ex)[:80]}
            continue
        settle_gpu(plan, Bs, Cs, torch, 100.0)  # as rocSPARSE's 300 untimed launches: past the idle clock
        ms = event_ms(plan, Bs, Cs, args.search_reps, torch)
        tried[key] = {"kernel": kernel_label(plan.info()), "kernel_ms": round(ms, 5)}
        if best32 is None or ms < best32[0]:
            best32 = (ms, key, tried[key]["kernel"])
        plan.free()
        del Bs, Cs
        torch.cuda.empty_cache()
    ms32 = best32[0]
    ours32 = flops / (ms32 * 1e-3) / 1e9
    res["rocsparse"].update({"ours_f32_gflops": round(ours32, 1), "ours_f32_kernel_ms": round(ms32, 5),
                             "ours_f32_plan": best32[1], "ours_f32_kernel": best32[2], "ours_f32_search": tried})
    if rs32:
        res["speedup_vs_rocsparse_f32"] = round(ours32 / rs32["gflops"], 3)
    return res


if __name__ == "__main__":
    main()
