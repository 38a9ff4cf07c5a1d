#!/bin/bash
# general-engine configs (tools/exp_gen.py) on the default build and on variant builds under siddhi-1_amd/
#   tools/gpu_libvar.sh "C3_min1 C4 C4_deep" lib_a lib_b ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CFGS=$1; shift
for v in default "$@"; do
  echo "== $v $(date +%T)"
  if [[ $v != default ]]; then export SG_HIP_LIBRARY=siddhi-1_amd/$v/libsiddhi_gpu.so; fi
  timeout -k 10 400 python tools/exp_gen.py $CFGS > gpurun_out/libvar_$v.log 2>&1 || { tail -20 gpurun_out/libvar_$v.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/libvar_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['config'], '%.3e'%d['value'], round(d['ms_per_step'],3), d['roofline']['kernel_ms_per_step'])"
done
