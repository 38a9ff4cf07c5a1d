#!/bin/bash
# General engine with several keys per lane: the general-engine GPU suites, then the bench's C3/C4 lines
# with one key per lane (GEN_KPL=1) and with the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r02m}
echo "== tests $(date +%T)"
timeout -k 10 700 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_baseline_configs.py tests/test_gpu_edges.py tests/test_gpu_engine_reuse.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/kpl_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/kpl_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/kpl_tests_$TAG.log
for v in 1 0; do
  echo "== bench kpl=$v $(date +%T)"
  if [[ $v == 1 ]]; then export GEN_KPL=1; else unset GEN_KPL; fi
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/kpl_$v.json 2> gpurun_out/kpl_$v.err || { tail -20 gpurun_out/kpl_$v.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/kpl_$v.json').read().strip().splitlines()[-1])
print('kpl=$v', {k:('%.3e'%x['value'], round(x['ms_per_step'],3), x['roofline']['kernel_ms_per_step']) for k,x in d['other_configs'].items()})"
done
