#!/bin/bash
cd ${GRAFT_REPO_ROOT}
# bench.py default line at several --steps / --warmup (C2 and its north_star object); the first 20/5 run is the driver command
mkdir -p gpurun_out/${TAG:-r05x}
for sw in "20 5" "200 20" "100 10" "20 5"; do
  set -- $sw
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps $1 --warmup $2 --no-cpu --no-rocsparse > gpurun_out/${TAG:-r05x}/b_$1_$2.log 2>&1 || exit 1
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/${TAG:-r05x}/b_$1_$2.log') if l.startswith('{')][-1]
ns=d['north_star']
print('steps $1 warmup $2: c2', d['ms_per_step'], d['config']['plan'], 'ns', ns['ms_per_step'], ns['steps'], ns['warmup'], ns['roofline']['frac'])"
done
