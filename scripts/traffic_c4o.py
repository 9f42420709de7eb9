"""profiles/traffic_c4o.json from scripts/traffic_c4o.sh: HBM bytes per SpMM launch of the com-Orkut
stand-in, summed over the launch's kernels (k_permute_rows + k_merge_path, or with MP_COL_PARTS=P
k_permute_rows + P x k_merge_path + k_add_parts).  FETCH_SIZE x2 (gfx950 streaming-read
undercount) and WRITE_SIZE, both KiB, from separate passes; per kernel the mean over its
dispatches times its dispatches per launch.  usage: traffic_c4o.py <dir> <out json>"""
import csv
import glob
import json
import os
import sys

ALG = 2083887320  # nnz (4 + 4) + (M + 1) 4 + K N 4 + M N 4, fp32 N = 8
root, out = sys.argv[1], sys.argv[2]


def per_kernel(d, counter):
    per = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")) + glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "gsk::" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("gsk::")[1].split("<")[0]
            per.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
            per[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


res = {"algorithmic_bytes_per_launch": ALG, "variants": {}}
for tag, plan, parts in (("p0", "merge_path(2048,1)", 1), ("p4", "merge_path(1024,1) MP_COL_PARTS=4", 4)):
    fe, nf = per_kernel(os.path.join(root, f"{tag}_FETCH_SIZE"), "FETCH_SIZE")
    wr, _ = per_kernel(os.path.join(root, f"{tag}_WRITE_SIZE"), "WRITE_SIZE")
    kern = {}
    total = 0
    for k in fe:
        mult = parts if k == "k_merge_path" else 1
        rb, wb = int(fe[k] * 1024 * 2 * mult), int(wr.get(k, 0.0) * 1024 * mult)
        kern[k] = {"dispatches_per_launch": mult, "hbm_read_bytes": rb, "hbm_write_bytes": wb, "dispatches_seen": nf[k]}
        total += rb + wb
    res["variants"][plan] = {"hbm_bytes_per_launch": total, "traffic_over_algorithmic": round(total / ALG, 3), "kernels": kern}
main = res["variants"]["merge_path(2048,1)"]
res.update({"kernel": "k_merge_path", "plan": "merge_path(2048,1)", "hbm_bytes_per_launch": main["hbm_bytes_per_launch"],
            "traffic_over_algorithmic": main["traffic_over_algorithmic"],
            "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes; includes Infinity-Cache hits",
            "note": "r06fin: the com-Orkut stand-in per SpMM launch (k_permute_rows + the merge-path passes + k_add_parts); "
                    "the MP_COL_PARTS=4 variant (one pass per column partition) moves about half the bytes at an even time"})
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({p: v["traffic_over_algorithmic"] for p, v in res["variants"].items()}))
