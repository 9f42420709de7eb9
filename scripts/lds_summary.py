"""Per-kernel averages of an LDS --pmc pass (scripts/lds_pmc.sh) over the last 20 dispatches of
each matrix-core kernel.  The bank-conflict share is SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
(extra cycles over all LDS-array cycles, same unit).  usage: lds_summary.py <run dir>..."""
import collections
import csv
import sys

for d in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f"{d}/p_counter_collection.csv")):
        if "mfma" in r["Kernel_Name"]:
            per[(r["Kernel_Name"], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    by_k = collections.defaultdict(list)
    for (k, did), c in sorted(per.items(), key=lambda kv: kv[0][1]):
        by_k[k].append(c)
    for k, lst in by_k.items():
        last = lst[-20:]
        avg = {n: sum(x[n] for x in last) / len(last) for n in last[0]}
        share = avg["SQ_LDS_BANK_CONFLICT"] / max(1.0, avg["SQ_LDS_IDX_ACTIVE"])
        print(f"{d} {k} dispatches={len(lst)} " + " ".join(f"{n}={v:.0f}" for n, v in sorted(avg.items()))
              + f" bank_conflict_share={share:.3f}")
