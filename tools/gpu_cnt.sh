#!/bin/bash
# counting-sequence register-window kernel: its parity tests, the general / baseline suites, then C3 timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r03c}
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_count_window.py \
    > gpurun_out/cnt_tests_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/cnt_tests_$TAG.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/cnt_tests_$TAG.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_general.py \
    tests/test_gpu_baseline_configs.py tests/test_gpu_state_doc.py tests/test_gpu_snapshot.py tests/test_gpu_purge.py \
    tests/test_gpu_absent_window.py > gpurun_out/cnt_tests2_$TAG.log 2>&1 || { tail -40 gpurun_out/cnt_tests2_$TAG.log; exit 1; }
tail -2 gpurun_out/cnt_tests2_$TAG.log
echo "== timing $(date +%T)"
SG_EXP_STEPS=4 timeout -k 10 300 python tools/exp_gen.py C3 C3_min1 > gpurun_out/cnt_exp_$TAG.log 2>&1 || { tail -20 gpurun_out/cnt_exp_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/cnt_exp_$TAG.log | cut -c1-300
