# round end: the whole -m gpu suite, then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_full.log 2>&1 || { tail -20 gpurun_out/gpu_full.log; exit 1; }
tail -2 gpurun_out/gpu_full.log
timeout -k 10 800 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
