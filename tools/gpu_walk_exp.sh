#!/bin/bash
# The staged pass walking the key-sorted payload in HBM (SGX_GLB_WALK, no LDS region: occupancy bound by
# VGPRs) against the LDS-staged walk, C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in lds glb; do
  echo "== $v $(date +%T)"
  if [[ $v == glb ]]; then export SG_JIT_EXTRA="SGX_GLB_WALK=1" SGD_STAGE_CHUNKS=64; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/walk_$v.json 2> gpurun_out/walk_$v.err || { tail -20 gpurun_out/walk_$v.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/walk_$v.json').read().strip().splitlines()[-1])
print('$v', '%.3e'%d['value'], d['ms_per_step'], d['stages_ms_isolated'], d['roofline']['frac'], d['roofline']['isolated']['frac'])"
done
