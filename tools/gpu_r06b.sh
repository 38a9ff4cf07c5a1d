#!/bin/bash
# round-6 GPU check (quick): the GPU tests, the C2 bench and the general-engine legs named in $2 (no CPU legs)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TAG=${1:-r06}
LEGS=${2:-P3,C3}
TESTS=${3:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
SG_BENCH_DETAIL=gpurun_out/${TAG}_detail.json timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu --legs $LEGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
