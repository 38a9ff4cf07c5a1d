set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export SG_BENCH_DEVICE=0 SG_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4194304 --keys 262144 --no-cpu --no-extra > gpurun_out/bench2.log 2>&1 || { tail -40 gpurun_out/bench2.log; exit 1; }
tail -2 gpurun_out/bench2.log | cut -c1-600
