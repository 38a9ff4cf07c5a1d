#!/bin/bash
# absent-tail register-window kernels: their parity tests, the absent / timer / KAT suites, then C4 timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r03c}
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_absent_window.py \
    > gpurun_out/abs_tests_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/abs_tests_$TAG.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/abs_tests_$TAG.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_general.py \
    tests/test_gpu_baseline_configs.py tests/test_gpu_state_doc.py tests/test_gpu_snapshot.py tests/test_gpu_purge.py \
    tests/test_gpu_parity.py tests/test_gpu_projection.py > gpurun_out/abs_tests2_$TAG.log 2>&1 || { tail -40 gpurun_out/abs_tests2_$TAG.log; exit 1; }
tail -2 gpurun_out/abs_tests2_$TAG.log
echo "== timing $(date +%T)"
SG_EXP_STEPS=4 timeout -k 10 300 python tools/exp_gen.py C4 C4_deep > gpurun_out/abs_exp_$TAG.log 2>&1 || { tail -20 gpurun_out/abs_exp_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/abs_exp_$TAG.log | cut -c1-250
