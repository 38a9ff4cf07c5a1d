#!/bin/bash
# C2 bench main line under environment variants (no CPU leg, no C3/C4):
#   tools/gpu_bench_env.sh NAME="VAR=value VAR2=value" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%=*}; vars=${v#*=}
  env $vars timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/env_$name.json 2> gpurun_out/env_$name.err || { tail -20 gpurun_out/env_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/env_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['roofline'].get('isolated',{}).get('kernel_ms_per_launch'))"
done
