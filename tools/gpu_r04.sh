#!/bin/bash
# Round-4 GPU session: the tests named in $FIRST first (fail fast), then every -m gpu test, smoke, bench,
# a rocprofv3 kernel-trace summary of the bench.  Every GPU step under its own time limit, chained.
#   FIRST="tests/test_gpu_sharded.py" tools/gpu_r04.sh <tag> [skip-prof]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r04}
if [[ -n "$FIRST" ]]; then
  echo "== first $(date +%T)"
  timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/gpu_first_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_first_$TAG.log; exit 1; }
  tail -2 gpurun_out/gpu_first_$TAG.log
fi
echo "== tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 400 gpurun_out/bench_$TAG.json
[[ "$2" == "skip-prof" ]] && exit 0
echo "== prof $(date +%T)"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -3
