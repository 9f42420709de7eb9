"""Pretty-print gpurun_out/timeline.json (mfma_timeline.py output): per role and chunk,
ticks of work + ticks of waiting at the chunk's barrier (entry role: ticks to issue
its loads + ticks of its scatter)."""
import json
import sys

d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/timeline.json"))
print("total", d["total_med"])
for role in ("compute", "bload", "aload"):
    r = d[role]
    prev = r["staged0"]
    line = [f"{role:8s} staged0 {r['staged0']:.0f} |"]
    for j in range(9):
        if f"c{j}" not in r:
            break
        done, after = r[f"c{j}"]
        line.append(f"{done - prev:.0f}+{after - done:.0f}")
        prev = after
    print(" ".join(line))
