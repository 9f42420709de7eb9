"""HBM bytes per launch of one kernel from the FETCH_SIZE / WRITE_SIZE passes
(MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of wide streaming
reads on gfx950 -> x2; both counters are in KiB).  Writes profiles/<out>.json.
usage: traffic_summary.py <pmc dir> <kernel substring> <out json> [algorithmic bytes] [plan label]"""
import csv
import re
import glob
import json
import os
import sys

root, filt, out = sys.argv[1], sys.argv[2], sys.argv[3]
alg = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] else None
plan = sys.argv[5] if len(sys.argv) > 5 else None
vals = {}
for name in ("FETCH_SIZE", "WRITE_SIZE"):
    per = {}
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and filt in r["Kernel_Name"]:
                per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    vals[name] = sum(per.values()) / max(1, len(per))
    vals[name + "_dispatches"] = len(per)
fetch_b = vals["FETCH_SIZE"] * 1024 * 2
write_b = vals["WRITE_SIZE"] * 1024
# the kernel family (the bench matches on it): the filter may be a mangled instantiation
label = re.match(r"k_[a-z0-9_]+", filt).group(0) if re.match(r"k_[a-z0-9_]+", filt) else filt
res = {"kernel": label, "filter": filt, "plan": plan, "fetch_size_kib_raw": round(vals["FETCH_SIZE"], 1), "write_size_kib": round(vals["WRITE_SIZE"], 1),
       "dispatches": vals["FETCH_SIZE_dispatches"], "hbm_read_bytes_per_launch": int(fetch_b),
       "hbm_write_bytes_per_launch": int(write_b), "hbm_bytes_per_launch": int(fetch_b + write_b),
       "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes"}
if alg:
    res["algorithmic_bytes_per_launch"] = alg
    res["traffic_over_algorithmic"] = round((fetch_b + write_b) / alg, 3)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
