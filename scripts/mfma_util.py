#!/usr/bin/env python3
"""Matrix-core utilisation of a kernel from one rocprofv3 --pmc pass (SURVEY
§8d): usage mfma_util.py <pmc dir> <kernel substring> <out.json> <workload>
[mfma instructions per dispatch] [cycles per mfma] [plan label].

Counters (scripts/gpu_session.sh part `sq`): SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy cycles,
summed over every SIMD of the chip), GRBM_GUI_ACTIVE (GPU-busy cycles, summed over the 8 XCDs,
MI355X_MICROARCH.md DVFS item), SQ_WAVE_CYCLES / SQ_BUSY_CYCLES (context).
  mfma_util_grbm = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
i.e. the fraction of the kernel's busy cycles, per SIMD, in which its matrix pipe was busy.
GRBM_GUI_ACTIVE over-counts on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS
give-back: the implied clock reads 2.6-3.7 GHz here), so the figure reported first is the
pessimistic one, against the peak clock over the kernel's own duration:
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel ns x 2.4 GHz)
and the GRBM-based ratio beside it (mfma_util_grbm).  The busy counter is checked against the
analytic instruction count (n_mfma x cycles per MFMA) when that is given."""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict

SIMDS = 1024  # 256 CUs x 4 SIMDs
XCDS = 8


def main():
    d, kern, dst, wl = sys.argv[1:5]
    n_mfma = float(sys.argv[5]) if len(sys.argv) > 5 else None
    cyc = float(sys.argv[6]) if len(sys.argv) > 6 else None
    plan = sys.argv[7] if len(sys.argv) > 7 else None
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    assert per, f"no dispatch of {kern} in {d}"
    keys = list(per)
    med = {c: statistics.median(per[k][c] for k in keys) for c in per[keys[0]]}
    active = med["GRBM_GUI_ACTIVE"] / XCDS
    label = re.match(r"k_[a-z0-9_]+", kern).group(0) if re.match(r"k_[a-z0-9_]+", kern) else kern
    out = {"workload": wl, "kernel": label, "filter": kern, "plan": plan, "dispatches": len(keys), "counters_median": med,
           "kernel_ns_median": statistics.median(dur.values()),
           "clock_ghz_est": round(active / statistics.median(dur.values()), 3),
           "mfma_util": round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * statistics.median(dur.values()) * 2.4), 4),
           "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel ns x 2.4 GHz)",
           "mfma_util_grbm": round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (active * SIMDS), 4),
           "formula_grbm": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)"}
    if n_mfma and cyc:
        out["analytic"] = {"mfma_per_dispatch": n_mfma, "cycles_per_mfma": cyc,
                           "busy_cycles": n_mfma * cyc,
                           "counter_over_analytic": round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (n_mfma * cyc), 4)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
