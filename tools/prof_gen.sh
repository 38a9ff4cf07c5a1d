# general configs: timing of the current build against lib_base (the previous build), then a kernel trace of C3 + C4
set -e
cd $GRAFT_REPO_ROOT
export SG_EXP_STEPS=8
echo "== base"; SG_HIP_LIBRARY=siddhi-1_amd/lib_base/libsiddhi_gpu.so timeout -k 10 200 python tools/exp_gen.py C3 C4 C3_min1
echo "== new"; timeout -k 10 200 python tools/exp_gen.py C3 C4 C3_min1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/gen_prof -o gen -- python3 $GRAFT_REPO_ROOT/tools/exp_gen.py C3 C4 > $GRAFT_REPO_ROOT/gpurun_out/gen_prof.log 2>&1
