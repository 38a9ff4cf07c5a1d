#!/bin/bash
# layout experiment: the general configs on the default build and on the variant builds given
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/exp_gen.py > gpurun_out/exp_gen_default.log 2>&1 || { tail -20 gpurun_out/exp_gen_default.log; exit 1; }
cat gpurun_out/exp_gen_default.log
for v in "$@"; do
  SG_HIP_LIBRARY=siddhi-1_amd/$v/libsiddhi_gpu.so timeout -k 10 300 python tools/exp_gen.py > gpurun_out/exp_gen_$v.log 2>&1 || { tail -20 gpurun_out/exp_gen_$v.log; exit 1; }
  cat gpurun_out/exp_gen_$v.log
done
