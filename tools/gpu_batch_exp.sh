#!/bin/bash
# C2 step at several batch sizes (LDS per advance workgroup scales with the batch: occupancy vs the
# sort's fixed costs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for b in 8388608 12582912 16777216; do
  echo "== batch $b $(date +%T)"
  timeout -k 10 200 python bench.py --batch $b --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/batch_$b.json 2> gpurun_out/batch_$b.err || { tail -20 gpurun_out/batch_$b.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/batch_$b.json').read().strip().splitlines()[-1])
print('$b', '%.3e'%d['value'], d['ms_per_step'], d['stages_ms_isolated'], d['roofline']['frac'], d['roofline']['isolated']['frac'])"
done
