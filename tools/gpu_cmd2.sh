#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_multirank.py tests/test_broadcast.py tests/test_gpu_general.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1 || { tail -60 gpurun_out/t2.log; exit 1; }
tail -5 gpurun_out/t2.log
echo "== 2-rank bench rehearsal"
SG_BENCH_DEVICE=0 SG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4194304 --keys 1048576 \
   > gpurun_out/bench2.log 2>&1 || { tail -30 gpurun_out/bench2.log; exit 1; }
grep '"metric"' gpurun_out/bench2.log | cut -c1-600
