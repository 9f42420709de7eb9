"""HBM bytes of one C5 batch step from the FETCH_SIZE / WRITE_SIZE passes over a
--layers L run of bench.py --workload c5 with GS_BENCH_MARK=1 (K timed steps): the gsk::
dispatches between the two spin-kernel markers bench.py launches around the timed region
(bench.mark; ADVICE r04: no dispatch-count window), summed per file in dispatch order,
divided by K and by L, times the 48 layers of the batch.  The expected dispatch count is
asserted (K x L x 6 single launches, or the grouped launches' count when --group 1).
FETCH_SIZE x2 on gfx950 (MI355X_MICROARCH.md §HBM), KiB -> bytes.
usage: traffic_c5.py <pmc root> <layers> <timed steps> <out json> [dispatches per step]"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generalsparse_amd import batch as bt  # noqa: E402

root, layers, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
tot = {}
kinds = set()
per_step = int(sys.argv[5]) if len(sys.argv) > 5 else layers * len(bt.C5_SLOTS)
kind_re = re.compile(r"gsk(?:::|\d+)(k_[a-z0-9_]+?)(?:I|<|\()")
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    total, n = 0.0, 0
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per, nm = {}, {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                key = int(r["Dispatch_Id"])
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
                nm[key] = r["Kernel_Name"]
        marks = [k for k in sorted(per) if "spin_kernel" in nm[k]]
        if len(marks) < 2:
            continue
        timed = [k for k in sorted(per) if marks[0] < k < marks[1] and "gsk" in nm[k]]
        for key in timed:
            m = kind_re.search(nm[key])
            kinds.add(m.group(1) if m else nm[key])
        total += sum(per[k] for k in timed)
        n += len(timed)
    assert n == steps * per_step, f"{name}: {n} timed dispatches, expected {steps} x {per_step}"
    tot[name] = (total, n)
layer_read = tot["FETCH_SIZE"][0] * 1024 * 2 / steps / layers
layer_write = tot["WRITE_SIZE"][0] * 1024 / steps / layers
e, N = 2, 32
alg_layer = sum(bt.nnz_of_shape(k) * (e + 2) + (bt.C5_SHAPES[k][0] + 1) * 4 + bt.C5_SHAPES[k][1] * N * e +
                bt.C5_SHAPES[k][0] * N * e for k in bt.C5_SLOTS)
res = {"kernel": "+".join(sorted(kinds)), "layers_profiled": layers, "steps_profiled": steps,
       "dispatches": {"FETCH_SIZE": tot["FETCH_SIZE"][1], "WRITE_SIZE": tot["WRITE_SIZE"][1]},
       "hbm_read_bytes_per_layer": int(layer_read), "hbm_write_bytes_per_layer": int(layer_write),
       "hbm_bytes_per_step": int((layer_read + layer_write) * 48), "algorithmic_bytes_per_step": alg_layer * 48,
       "traffic_over_algorithmic": round((layer_read + layer_write) / alg_layer, 3),
       "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
