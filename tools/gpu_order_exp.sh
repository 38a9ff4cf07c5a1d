#!/bin/bash
# Ordering-stage ablation (SG_ORDER_EXP=1: no raw_e1 gather, wrong results): kernel trace of the C2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for x in 0 1; do
  echo "== exp $x $(date +%T)"
  SG_ORDER_EXP=$x timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/oexp_$x -o run --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra > gpurun_out/oexp_$x.log 2>&1 || { tail -20 gpurun_out/oexp_$x.log; exit 1; }
done
