#!/bin/bash
# Round-end validation: every -m gpu test, smoke, the default bench line, a C2-only kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r02p}
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
print('%.3e'%d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['isolated']['frac'], {k:'%.3e'%d[k]['value'] for k in ('pcie_inclusive','output_inclusive','api_inclusive','api_columnar') if k in d}, {k:'%.3e'%x['value'] for k,x in d['other_configs'].items()})"
echo "== prof $(date +%T)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extra > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -3
