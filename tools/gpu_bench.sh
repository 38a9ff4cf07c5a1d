#!/bin/bash
# Bench + rocprofv3 kernel-trace summary only (tests already green):  tools/gpu_bench.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r02}
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 600 gpurun_out/bench_$TAG.json
echo "== prof $(date +%T)"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*kernel_stats.csv'
