set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/exp_c2.py 4 "prof:SG_PROF=1;SG_JIT_EXTRA=SGX_PROF=1" "noloop:SG_JIT_EXTRA=SGX_NO_LOOP=1" "it4:SG_JIT_EXTRA=SGX_MAX_IT=4" "noboth:SG_JIT_EXTRA=SGX_NO_TDESC=1,SGX_NO_RAW=1" > gpurun_out/exp1.log 2>&1 || { tail -30 gpurun_out/exp1.log; exit 1; }
grep "variant\|SG_PROF" gpurun_out/exp1.log
bash tools/pmc_c2.sh
