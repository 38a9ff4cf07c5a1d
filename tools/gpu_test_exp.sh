#!/bin/bash
# GPU tests (all -m gpu) then the C2 advance-kernel sweep:  tools/gpu_test_exp.sh <tag> [variants...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-x}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python tools/exp_c2.py 5 "$@" > gpurun_out/exp_$TAG.log 2>&1 || { tail -30 gpurun_out/exp_$TAG.log; exit 1; }
grep variant gpurun_out/exp_$TAG.log
