"""Summary of scripts/pmc_bytes.sh: per dispatch of the kernels matching a filter, the L2 ->
fabric read requests by size (32/64/128 B) and the bytes they carry, L2 hit rate, the
DRAM-bound share, write requests and TCP->TCC read requests.
usage: pmc_bytes.py <dir> <kernel substring> [algorithmic read bytes] [out json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, filt = sys.argv[1], sys.argv[2]
alg = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "-" else None
out = sys.argv[4] if len(sys.argv) > 4 else None
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d in per.values():
        for c, v in d.items():
            vals[c].append(v)
m = {c: sum(v) / len(v) for c, v in vals.items()}
n = {c: len(v) for c, v in vals.items()}
g = lambda k: m.get(k, m.get(k.replace("_sum", ""), 0.0))
rq, r32, r64, r128 = g("TCC_EA0_RDREQ_sum"), g("TCC_EA0_RDREQ_32B_sum"), g("TCC_EA0_RDREQ_64B_sum"), g("TCC_EA0_RDREQ_128B_sum")
res = {"kernel": filt, "dispatches": n, "counters_per_dispatch": {k: round(v, 1) for k, v in sorted(m.items())}}
rd = 32 * r32 + 64 * r64 + 128 * r128
res["read_bytes_by_request_size"] = int(rd)
res["read_requests_unsized"] = round(rq - r32 - r64 - r128, 1)
res["fetch_size_expression_bytes"] = int(g("TCC_BUBBLE_sum") * 128 + (rq - g("TCC_BUBBLE_sum") - r32) * 64 + r32 * 32)
hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
if hit + miss:
    res["l2_hit_rate"] = round(hit / (hit + miss), 4)
if rq:
    res["dram_share_of_requests"] = round(g("TCC_EA0_RDREQ_DRAM_sum") / rq, 4)
if alg:
    res["algorithmic_read_bytes"] = alg
    res["read_over_algorithmic"] = round(rd / alg, 3)
print(json.dumps(res, indent=1))
if out:
    json.dump(res, open(out, "w"), indent=1)
