#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, a rocprofv3 kernel-trace summary of the bench.
# Every GPU step has its own time limit and the chain stops at the first failure.
#   tools/gpu_round.sh [all|tests|smoke|bench|prof] [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEP=${1:-all}
TAG=${2:-r01}
run() { echo "== $1 $(date +%T)"; shift; "$@"; }
if [[ $STEP == all || $STEP == tests ]]; then
  run tests timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [[ $STEP == all || $STEP == slow ]]; then
  run slow timeout -k 10 600 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 500 --timeout-method thread \
      > gpurun_out/gpu_slow.log 2>&1 || { tail -60 gpurun_out/gpu_slow.log; exit 1; }
  tail -3 gpurun_out/gpu_slow.log
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  run smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run bench timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  export TMPDIR=/tmp
  run prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
      -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
  tail -2 gpurun_out/prof_$TAG.log
  find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -3
fi
