#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="tests/test_gpu_edges.py::test_ragged_and_empty_batches"
timeout -k 10 200 python -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
SG_JIT_EXTRA=SGX_NO_DEAL=1 timeout -k 10 200 python -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
SGD_STAGE_CHUNKS=8000 timeout -k 10 200 python -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
SGD_REG_SLOTS=16 timeout -k 10 200 python -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
