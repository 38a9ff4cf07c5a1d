#!/bin/bash
# round 3: fan-out tests, C2 parity with the branchless window, then the A/B timing of the window variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py \
    tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_projection.py > gpurun_out/r03f_tests.log 2>&1 \
    || { tail -40 gpurun_out/r03f_tests.log; exit 1; }
tail -2 gpurun_out/r03f_tests.log
echo "== A/B $(date +%T)"
SG_HIP_LIBRARY=siddhi-1_amd/lib_exp/libsiddhi_gpu.so timeout -k 10 300 python tools/exp_c2.py 4 \
    "branchy:SG_JIT_EXTRA=SGX_BRANCHLESS=0" "branchless2:SG_JIT_EXTRA=SGX_BRANCHLESS=1" > gpurun_out/r03f_ab.log 2>&1 \
    || { tail -20 gpurun_out/r03f_ab.log; exit 1; }
cat gpurun_out/r03f_ab.log | cut -c1-300
