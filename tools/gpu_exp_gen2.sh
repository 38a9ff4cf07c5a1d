#!/bin/bash
# general-engine configs under alternative library builds:  tools/gpu_exp_gen2.sh lib_a lib_b ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for l in default "$@"; do
  if [ "$l" = default ]; then unset SG_HIP_LIBRARY; else export SG_HIP_LIBRARY=$PWD/siddhi-1_amd/$l/libsiddhi_gpu.so; fi
  SG_EXP_STEPS=3 timeout -k 10 300 python tools/exp_gen.py C3_min1 C4 C4_deep > gpurun_out/expgen2_$l.log 2>&1 || { tail -20 gpurun_out/expgen2_$l.log; exit 1; }
  python3 -c "
import json
for x in open('gpurun_out/expgen2_$l.log'):
    if x.startswith('{'):
        d=json.loads(x); print('$l', d['config'], '%.4g'%d['value'])
"
done
