"""Summarise rocprofv3 csv outputs of pmc_sq.sh: per kernel, mean duration and
mean counter value per dispatch (diagnostic only)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if filt in r["Name"]:
            print(f"{r['Name'][:70]:70s} calls={r['Calls']} avg_ns={float(r['AverageNs']):.0f}")
cnt = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), d in per.items():
        for c, v in d.items():
            cnt[k][c].append(v)
for k, d in cnt.items():
    print(k[:90])
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
