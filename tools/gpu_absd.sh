#!/bin/bash
# wave-per-key deep absent kernels: the absent parity suites, then C4 / C4_deep / C4_deep_state timings (A/B)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r03h}
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_absent_window.py \
    > gpurun_out/absd_tests_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/absd_tests_$TAG.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/absd_tests_$TAG.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_general.py \
    tests/test_gpu_baseline_configs.py tests/test_gpu_state_doc.py tests/test_gpu_snapshot.py tests/test_gpu_purge.py \
    tests/test_gpu_sharded.py > gpurun_out/absd_tests2_$TAG.log 2>&1 || { tail -40 gpurun_out/absd_tests2_$TAG.log; exit 1; }
tail -2 gpurun_out/absd_tests2_$TAG.log
echo "== timing $(date +%T)"
SG_EXP_STEPS=4 timeout -k 10 400 python tools/exp_gen.py C4 C4_deep C4_deep_state > gpurun_out/absd_exp_$TAG.log 2>&1 || { tail -20 gpurun_out/absd_exp_$TAG.log; exit 1; }
SG_NO_ABSD=1 SG_EXP_STEPS=4 timeout -k 10 600 python tools/exp_gen.py C4_deep > gpurun_out/absd_exp_off_$TAG.log 2>&1 || { tail -20 gpurun_out/absd_exp_off_$TAG.log; exit 1; }
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/absd_exp*_r03h.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d["config"], round(d["value"] / 1e6, 2), "M ev/s", round(d["ms_per_step"], 3), "ms",
                  d["roofline"]["counters_per_step"])
PY
