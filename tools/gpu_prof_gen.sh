#!/bin/bash
# per-config kernel-trace summaries of the general-engine configs:  tools/gpu_prof_gen.sh <tag> [configs...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp SG_EXP_STEPS=3
TAG=${1:-r03}
shift
for c in "${@:-C3_min1 C4 C4_deep}"; do
  for cc in $c; do
    echo "== $cc $(date +%T)"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$cc -o run --output-format csv \
        -- python3 tools/exp_gen.py $cc > gpurun_out/prof_${TAG}_$cc.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}_$cc.log; exit 1; }
    grep -v "^config" gpurun_out/prof_${TAG}_$cc.log | tail -1 | cut -c1-300
  done
done
