#!/bin/bash
# stream priorities of the two-stream batch pipeline (SG_STREAM_PRIO), C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for p in none g m; do
  echo "== prio $p $(date +%T)"
  SG_STREAM_PRIO=$p timeout -k 10 200 python bench.py --steps 32 --warmup 3 --no-cpu --no-extra > gpurun_out/prio_$p.json 2> gpurun_out/prio_$p.err || { tail -20 gpurun_out/prio_$p.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/prio_$p.json').read().strip().splitlines()[-1])
print('$p', '%.3e'%d['value'], round(d['ms_per_step'],3), d['stages_ms_per_step'], round(d['roofline']['frac'],4))"
done
