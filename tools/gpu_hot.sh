# hot-key pipeline: its GPU tests, then the C2 variants' stage times (current build vs lib_base)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_hotkeys.py tests/test_gpu_grouping.py > gpurun_out/hot_tests.log 2>&1 || { tail -30 gpurun_out/hot_tests.log; exit 1; }
tail -2 gpurun_out/hot_tests.log
echo "== base"; SG_HIP_LIBRARY=siddhi-1_amd/lib_base/libsiddhi_gpu.so timeout -k 10 200 python tools/exp_variants.py 24 12 zipf walk
echo "== new"; timeout -k 10 200 python tools/exp_variants.py 24 12 zipf walk uniform
