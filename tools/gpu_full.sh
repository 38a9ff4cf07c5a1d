# the whole -m gpu suite, then the C2 / C3 / C4 legs of the bench (short), on the box
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_full.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_full.log
exit $rc
