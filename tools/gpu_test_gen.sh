#!/bin/bash
# GPU tests (all -m gpu) then the general-engine configs (C3_min1, C4, C4_deep):  tools/gpu_test_gen.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python tools/exp_gen.py C3 C3_min1 C4 C4_deep > gpurun_out/expgen_$TAG.log 2>&1 || { tail -30 gpurun_out/expgen_$TAG.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/expgen_$TAG.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], '%.4g'%d['value'], d.get('ms_per_step'))
"
