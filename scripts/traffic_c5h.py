"""HBM traffic per launch of every (shape, candidate plan) the headline layer's plan search
(bench.py --workload c5h) can pick: `run` builds one shape's matrix with one candidate and
launches it `steps` times; run it under rocprofv3 --pmc FETCH_SIZE and again under --pmc
WRITE_SIZE (separate passes, one process per combination: scripts/gpu_traffic_c5h.sh), then
`summarize` sums each combination's dispatches and divides by the steps (FETCH_SIZE x2 on
gfx950, MI355X_MICROARCH.md §HBM).  bench.py's c5h line sums the entries of the plans its
search chose over the layer's six slots.
usage: traffic_c5h.py list | run <shape> <cand> <steps> | summarize <pmc root> <steps> <out json>"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N, SP = 32, 0.7


def key(c):
    """the plan key bench.py's search_shapes reports"""
    return "%s(%d,%d)%s" % (c[0], c[1], c[2], "".join(f" {a}={b}" for a, b in c[3].items()))


def alg_launch(k):
    from generalsparse_amd import batch as bt
    m, n = bt.C5_SHAPES[k]
    return bt.nnz_of_shape(k, SP) * 4 + (m + 1) * 4 + n * N * 2 + m * N * 2


def run(shape, ci, steps):
    import torch
    import generalsparse_amd as gsa
    from generalsparse_amd import batch as bt
    from generalsparse_amd import datasets as ds
    dev = torch.device("cuda:0")
    m, n = bt.C5_SHAPES[shape]
    row, col, val = ds.pruned_weight(m, n, SP, bt.shape_seed(0, shape))
    plan = bt.build_plan(gsa, m, n, row, col, val, N, bt.shape_candidates(shape)[ci], 0)
    b = torch.randn((n, N), device=dev, dtype=torch.float16)
    c = torch.empty((m, N), device=dev, dtype=torch.float16)
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(steps):
        plan.spmm_raw(b.data_ptr(), c.data_ptr(), N, 0, stream)
    torch.cuda.synchronize()
    print(shape, key(bt.shape_candidates(shape)[ci]), plan.info()["device_kernel"])
    plan.free()


def summarize(root, steps, out):
    from generalsparse_amd import batch as bt
    res = {"N": N, "sparsity": SP, "steps_profiled": steps,
           "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes", "per_launch": {}}
    for shape in bt.C5_SHAPES:
        for ci, cand in enumerate(bt.shape_candidates(shape)):
            tot = {}
            for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
                per = {}
                for f in glob.glob(os.path.join(root, f"{sub}_{shape}_{ci}", "**", "*counter_collection.csv"),
                                   recursive=True):
                    for r in csv.DictReader(open(f)):
                        if r["Counter_Name"] == name and "gsk" in r["Kernel_Name"]:
                            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
                tot[name] = (sum(per.values()), len(per))
            if not tot["FETCH_SIZE"][1] or not tot["WRITE_SIZE"][1]:
                continue
            rd = tot["FETCH_SIZE"][0] * 1024 * 2 / steps
            wr = tot["WRITE_SIZE"][0] * 1024 / steps
            alg = alg_launch(shape)
            res["per_launch"].setdefault(shape, {})[key(cand)] = {
                "dispatches": tot["FETCH_SIZE"][1], "hbm_read_bytes": int(rd), "hbm_write_bytes": int(wr),
                "hbm_bytes": int(rd + wr), "algorithmic_bytes": alg, "traffic_over_algorithmic": round((rd + wr) / alg, 3)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "list":
        from generalsparse_amd import batch as bt
        print(" ".join(f"{k}:{i}" for k in bt.C5_SHAPES for i in range(len(bt.shape_candidates(k)))))
    elif sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        summarize(sys.argv[2], int(sys.argv[3]), sys.argv[4])
