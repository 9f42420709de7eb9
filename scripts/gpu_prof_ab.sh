#!/bin/bash
# kernel stats of one workload under several library builds (GS_LIBRARY A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out/pab
WL=${WL:-c4}
for v in ${LIBS:-main}; do
  [ "$v" = main ] && v=""
  GS_LIBRARY=$PWD/generalsparse_amd/libgeneralsparse$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab/$WL$v -o p -- python3 bench.py --workload $WL --steps 100 --warmup 10 --no-cpu --no-rocsparse ${BARGS} > gpurun_out/pab/$WL$v.log 2>&1
  python3 - <<PY
import csv, json
for r in csv.DictReader(open("gpurun_out/pab/$WL$v/p_kernel_stats.csv")):
    if "gsk" in r["Name"]: print("lib$v", r["Name"][:60], r["Calls"], r["AverageNs"])
d=[json.loads(l) for l in open("gpurun_out/pab/$WL$v.log") if l.startswith("{")][-1]
print("lib$v bench", d["value"], d["roofline"]["kernel_ms"])
PY
done
