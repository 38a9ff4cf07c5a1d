# the whole -m gpu suite, then the C2 variants' stage times, on the box
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_full.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_full.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$SG_FULL_EXP" ]; then timeout -k 10 200 python tools/exp_variants.py 24 8 walk uniform zipf > gpurun_out/exp_after_full.log 2>&1; fi
