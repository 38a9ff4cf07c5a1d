#!/bin/bash
# round-6 GPU check: the new chain-kernel tests, the whole -m gpu suite, then the C2 bench (and an A/B with the
# hot-key detection off)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TAG=${1:-r06}
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain_window.py -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_chain.log 2>&1 || { tail -40 gpurun_out/${TAG}_chain.log; exit 1; }
tail -3 gpurun_out/${TAG}_chain.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
SG_BENCH_DETAIL=gpurun_out/${TAG}_c2_detail.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || exit 1
cat gpurun_out/${TAG}_c2.json
SG_HOT_MIN=0 SG_BENCH_DETAIL=gpurun_out/${TAG}_c2_nohot_detail.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu > gpurun_out/${TAG}_c2_nohot.json 2> gpurun_out/${TAG}_c2_nohot.err || exit 1
cat gpurun_out/${TAG}_c2_nohot.json
