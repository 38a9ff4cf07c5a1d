#!/bin/bash
# C2 bench main line under JIT variants (no CPU leg, no C3/C4):  tools/gpu_bench_ab.sh NAME=SG_JIT_EXTRA ...
# (SG_JIT_EXTRA: space-separated NAME=VALUE macro definitions for the hipRTC compile of p2_jit.hip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%=*}; extra=${v#*=}
  SG_JIT_EXTRA=$extra timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -20 gpurun_out/ab_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['roofline'].get('isolated',{}).get('kernel_ms_per_launch'))"
done
