#!/bin/bash
# every -m gpu test, smoke, then the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r02o}
echo "== tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1])
print('%.3e'%d['value'], d['ms_per_step'], d['roofline']['frac'], {k:'%.3e'%d[k]['value'] for k in ('pcie_inclusive','output_inclusive','api_inclusive','api_columnar') if k in d})"
