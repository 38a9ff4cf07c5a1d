#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_projection.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1 || { tail -60 gpurun_out/t3.log; exit 1; }
tail -3 gpurun_out/t3.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { tail -30 gpurun_out/bench3.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench3.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print(json.dumps(d['output_inclusive'])); print(json.dumps(d['cpu_baseline']))
for k,v in d['other_configs'].items(): print(k, v['value'])
"
