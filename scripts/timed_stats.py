#!/usr/bin/env python3
"""Per-kernel statistics of the TIMED regions of a bench.py run under
`rocprofv3 --kernel-trace` with GS_BENCH_MARK=1.

bench.py launches one tiny spin kernel (torch.cuda._sleep) right before the first and right after the last
timed launch of each measured region (bench.mark); this script keeps only the dispatches
strictly between each pair of markers, so the plan search's launches of the same kernels
are not averaged in.  usage: timed_stats.py <rocprof output dir> <out.csv> [expected
dispatches per region, comma separated]"""
import csv
import glob
import os
import statistics
import sys

MARK = "spin_kernel"


def regions(rows):
    """[(dispatches between marker 2i and marker 2i+1)] in dispatch order"""
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        if MARK in r["Kernel_Name"]:
            if cur is None:
                cur = []
            else:
                out.append(cur)
                cur = None
        elif cur is not None:
            cur.append(r)
    return out


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def main():
    d, dst = sys.argv[1], sys.argv[2]
    expect = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    regs = regions(rows)
    if expect is not None:
        got = [len(r) for r in regs]
        assert got == expect, f"dispatches per timed region {got}, expected {expect}"
    with open(dst, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["region", "Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "RegionSpanNs"])
        for i, reg in enumerate(regs):
            span = (max(int(r["End_Timestamp"]) for r in reg) - min(int(r["Start_Timestamp"]) for r in reg)) if reg else 0
            by = {}
            for r in reg:
                by.setdefault(short(r["Kernel_Name"]), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for name, ds in sorted(by.items(), key=lambda x: -sum(x[1])):
                w.writerow([i, name, len(ds), sum(ds), round(statistics.mean(ds), 1), min(ds), max(ds), span])
                print(f"region {i}: {name[:70]:70s} calls {len(ds):4d} avg {statistics.mean(ds) / 1e3:9.2f} us "
                      f"min {min(ds) / 1e3:8.2f} max {max(ds) / 1e3:8.2f}  (region span {span / 1e3:.1f} us)")


if __name__ == "__main__":
    main()
