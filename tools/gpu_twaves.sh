#!/bin/bash
# timer-sweep occupancy (GEN_TWAVES builds under siddhi-1_amd/lib_t*) on C4 / C4_deep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in default lib_t2 lib_t3; do
  echo "== $v $(date +%T)"
  if [[ $v != default ]]; then export SG_HIP_LIBRARY=siddhi-1_amd/$v/libsiddhi_gpu.so; fi
  timeout -k 10 300 python tools/exp_gen.py C4 C4_deep > gpurun_out/twaves_$v.log 2>&1 || { tail -20 gpurun_out/twaves_$v.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/twaves_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['config'], '%.3e'%d['value'], round(d['ms_per_step'],3), d['roofline']['kernel_ms_per_step'])"
done
