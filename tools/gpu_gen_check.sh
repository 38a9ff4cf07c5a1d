#!/bin/bash
# general-engine suites (KATs on the device, state documents, snapshots, baseline sizes) + the general configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== tests $(date +%T)"
timeout -k 10 800 python -u -m pytest tests/test_gpu_general.py tests/test_gpu_state_doc.py tests/test_gpu_snapshot.py tests/test_gpu_baseline_configs.py tests/test_gpu_parity.py tests/test_gpu_projection.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gen_check.log 2>&1 || { tail -60 gpurun_out/gen_check.log; exit 1; }
tail -2 gpurun_out/gen_check.log
echo "== configs $(date +%T)"
timeout -k 10 400 python tools/exp_gen.py C3_min1 C4 C4_deep > gpurun_out/gen_check_cfg.log 2>&1 || { tail -20 gpurun_out/gen_check_cfg.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/gen_check_cfg.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], '%.3e'%d['value'], round(d['ms_per_step'],3), d['roofline']['kernel_ms_per_step'])"
