set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/exp_c2.py 4 "r12:SGD_REG_SLOTS=12" "r12noloop:SGD_REG_SLOTS=12;SG_JIT_EXTRA=SGX_NO_LOOP=1" "r12st512:SGD_REG_SLOTS=12;SGD_STAGE_CHUNKS=512" "r12noloop_st512:SGD_REG_SLOTS=12;SGD_STAGE_CHUNKS=512;SG_JIT_EXTRA=SGX_NO_LOOP=1" > gpurun_out/exp1.log 2>&1 || { tail -30 gpurun_out/exp1.log; exit 1; }
grep variant gpurun_out/exp1.log
