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
give-back: GRBM_GUI_ACTIVE / 8 / duration reads 2.6-3.8 GHz on these ~13-70 us dispatches, above
the 2.4 GHz the chip can run), so every figure divides by the PMC pass's own
dispatch duration (Start / End timestamps of the counter-collection record, not the duration of
another run) and a clock that is at most the 2.4 GHz peak:
  clock_ghz_est  = min(2.4, GRBM_GUI_ACTIVE / 8 / dispatch ns)   (the raw quotient is kept as
                   clock_ghz_grbm_raw)
  mfma_util      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dispatch ns x 2.4 GHz)      (vs peak)
  mfma_util_at_clock_est = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dispatch ns x clock_ghz_est)
Both equal when GRBM reads high (clock_ghz_est = 2.4).  The busy counter is checked against the
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
PEAK_GHZ = 2.4  # MI355X peak engine clock


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
    ns = statistics.median(dur.values())  # the PMC pass's own dispatch durations
    raw = active / ns
    clk = min(PEAK_GHZ, raw)
    label = re.match(r"k_[a-z0-9_]+", kern).group(0) if re.match(r"k_[a-z0-9_]+", kern) else kern
    busy = med["SQ_VALU_MFMA_BUSY_CYCLES"]
    out = {"workload": wl, "kernel": label, "filter": kern, "plan": plan, "dispatches": len(keys), "counters_median": med,
           "kernel_ns_median": ns, "kernel_ns_source": "this PMC pass's dispatch timestamps",
           "clock_ghz_grbm_raw": round(raw, 3), "clock_ghz_est": round(clk, 3),
           "mfma_util": round(busy / (SIMDS * ns * PEAK_GHZ), 4),
           "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dispatch ns x 2.4 GHz)",
           "mfma_util_at_clock_est": round(busy / (SIMDS * ns * clk), 4),
           "formula_at_clock_est": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dispatch ns x min(2.4, GRBM_GUI_ACTIVE/8/ns))"}
    assert out["clock_ghz_est"] <= PEAK_GHZ
    if n_mfma and cyc:
        out["analytic"] = {"mfma_per_dispatch": n_mfma, "cycles_per_mfma": cyc,
                           "busy_cycles": n_mfma * cyc,
                           "counter_over_analytic": round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (n_mfma * cyc), 4)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
