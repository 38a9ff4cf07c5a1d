#!/bin/bash
# deep-absent chunked walk: its parity tests (against the per-event walk and the oracle), the absent / general
# suites, then C4 / C4_deep / C4_deep_state timings with the chunked walk and without (SG_NO_ABSD_CHUNK=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r04e}
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_absent_window.py \
    > gpurun_out/absd2_tests_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/absd2_tests_$TAG.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/absd2_tests_$TAG.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_general.py \
    tests/test_gpu_baseline_configs.py tests/test_gpu_state_doc.py tests/test_gpu_snapshot.py tests/test_gpu_sharded.py \
    > gpurun_out/absd2_tests2_$TAG.log 2>&1 || { tail -40 gpurun_out/absd2_tests2_$TAG.log; exit 1; }
tail -2 gpurun_out/absd2_tests2_$TAG.log
echo "== timing $(date +%T)"
SG_EXP_STEPS=4 timeout -k 10 400 python tools/exp_gen.py C4 C4_deep C4_deep_state > gpurun_out/absd2_exp_$TAG.log 2>&1 || { tail -20 gpurun_out/absd2_exp_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/absd2_exp_$TAG.log | cut -c1-200
SG_NO_ABSD_CHUNK=1 SG_EXP_STEPS=4 timeout -k 10 400 python tools/exp_gen.py C4 C4_deep C4_deep_state > gpurun_out/absd2_exp_serial_$TAG.log 2>&1 || { tail -20 gpurun_out/absd2_exp_serial_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/absd2_exp_serial_$TAG.log | cut -c1-200
