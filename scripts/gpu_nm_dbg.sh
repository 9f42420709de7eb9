set -e
mkdir -p gpurun_out/nm
for d in 0 1 2 0; do
  GS_NM_DEBUG=$d timeout -k 10 200 python3 -u scripts/time_nm.py 28672 7168 128 2000 > gpurun_out/nm/dbg$d.log 2>&1
  echo "dbg $d: $(tail -1 gpurun_out/nm/dbg$d.log)"
done
