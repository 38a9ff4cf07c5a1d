#!/bin/bash
# grid of the listed HBM pass (SG_HBM_GRID one-wave work-groups), C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for g in 2048 512 128; do
  echo "== grid $g $(date +%T)"
  SG_HBM_GRID=$g timeout -k 10 200 python bench.py --steps 32 --warmup 3 --no-cpu --no-extra > gpurun_out/hgrid_$g.json 2> gpurun_out/hgrid_$g.err || { tail -20 gpurun_out/hgrid_$g.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/hgrid_$g.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$g', '%.3e'%d['value'], round(d['ms_per_step'],3), round(r['kernel_ms_per_launch'],4), round(r['hbm_pass_ms_per_launch'],4), round(r['frac'],4), round(r['isolated']['kernel_ms_per_launch'],4))"
done
