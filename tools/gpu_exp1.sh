set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > gpurun_out/p2.log 2>&1 || { tail -40 gpurun_out/p2.log; exit 1; }
tail -2 gpurun_out/p2.log
timeout -k 10 600 python -u tools/exp_c2.py 4 "r10:SGD_REG_SLOTS=10" "r8:SGD_REG_SLOTS=8" "prof:SG_PROF=1;SG_JIT_EXTRA=SGX_PROF=1" > gpurun_out/exp1.log 2>&1 || { tail -30 gpurun_out/exp1.log; exit 1; }
grep "variant\|SG_PROF" gpurun_out/exp1.log
