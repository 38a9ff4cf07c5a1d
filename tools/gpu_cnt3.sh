#!/bin/bash
# the count kernel's logical AND pair: the count / general / baseline / state suites, then C3 / C3_min1 / C3_and
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r04j}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_count_window.py \
    tests/test_gpu_general.py tests/test_gpu_baseline_configs.py tests/test_gpu_state_doc.py tests/test_gpu_parity.py \
    tests/test_gpu_snapshot.py > gpurun_out/cnt3_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/cnt3_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/cnt3_tests_$TAG.log
SG_EXP_STEPS=4 timeout -k 10 300 python tools/exp_gen.py C3 C3_min1 C3_and > gpurun_out/cnt3_exp_$TAG.log 2>&1 || { tail -20 gpurun_out/cnt3_exp_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/cnt3_exp_$TAG.log | cut -c1-160
