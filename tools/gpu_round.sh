#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Every GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEP=${1:-all}
run() { echo "== $1"; shift; "$@"; }
if [[ $STEP == all || $STEP == tests ]]; then
  run tests timeout -k 10 600 python -m pytest tests -m "gpu and not slow" -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  run smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run bench timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
