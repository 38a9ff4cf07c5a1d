#!/bin/bash
# register-native records (GEN_W0_REG) of the count and absent register-window kernels: their parity tests,
# the fan-out seq-map test, the general / baseline / state suites, then C3 / C4 timings with the records and
# without (SG_NO_REC=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r04c}
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_count_window.py \
    tests/test_gpu_absent_window.py tests/test_gpu_sharded.py tests/test_gpu_multirank.py > gpurun_out/rec_tests_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/rec_tests_$TAG.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/rec_tests_$TAG.log
if [ -z "$QUICK" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_general.py \
    tests/test_gpu_baseline_configs.py tests/test_gpu_state_doc.py tests/test_gpu_snapshot.py tests/test_gpu_purge.py \
    > gpurun_out/rec_tests2_$TAG.log 2>&1 || { tail -40 gpurun_out/rec_tests2_$TAG.log; exit 1; }
tail -2 gpurun_out/rec_tests2_$TAG.log
fi
echo "== timing $(date +%T)"
SG_EXP_STEPS=4 timeout -k 10 400 python tools/exp_gen.py C3 C3_min1 C4 C4_deep > gpurun_out/rec_exp_$TAG.log 2>&1 || { tail -20 gpurun_out/rec_exp_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/rec_exp_$TAG.log | cut -c1-300
SG_NO_REC=1 SG_EXP_STEPS=4 timeout -k 10 400 python tools/exp_gen.py C3 C3_min1 C4 C4_deep > gpurun_out/rec_exp_blk_$TAG.log 2>&1 || { tail -20 gpurun_out/rec_exp_blk_$TAG.log; exit 1; }
grep -v "^config" gpurun_out/rec_exp_blk_$TAG.log | cut -c1-300
