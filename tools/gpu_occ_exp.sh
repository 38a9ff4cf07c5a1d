#!/bin/bash
# Occupancy of the staged advance pass: the same half-density C2 batch (2^23 events, 2^20 keys) with the
# LDS region at its natural size (~36 KB: 4 workgroups per CU) and forced to 70 KB (2 per CU) / 108 KB (1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for sc in 0 1100 1700; do
  echo "== stage $sc $(date +%T)"
  if [[ $sc == 0 ]]; then unset SGD_STAGE_CHUNKS; else export SGD_STAGE_CHUNKS=$sc; fi
  timeout -k 10 200 python bench.py --batch 8388608 --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/occ_$sc.json 2> gpurun_out/occ_$sc.err || { tail -20 gpurun_out/occ_$sc.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/occ_$sc.json').read().strip().splitlines()[-1])
print('$sc', '%.3e'%d['value'], d['ms_per_step'], d['stages_ms_isolated'], d['roofline'].get('hbm_pass_ms_per_launch'))"
done
