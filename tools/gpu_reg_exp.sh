#!/bin/bash
# register-window size of the staged pass (SGD_REG_SLOTS) on C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 8 10 12 14; do
  echo "== R=$r $(date +%T)"
  SGD_REG_SLOTS=$r timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/reg_$r.json 2> gpurun_out/reg_$r.err || { tail -20 gpurun_out/reg_$r.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/reg_$r.json').read().strip().splitlines()[-1])
print('R=$r', '%.3e'%d['value'], round(d['ms_per_step'],3), d['stages_ms_isolated'], d['roofline']['isolated'], d['work_per_step'].get('window_spills'))"
done
