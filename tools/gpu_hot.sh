# hot-key pipeline: its GPU tests, then the C2 variants' stage times
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_hotkeys.py tests/test_gpu_grouping.py tests/test_gpu_parity.py > gpurun_out/hot_tests.log 2>&1 || { tail -30 gpurun_out/hot_tests.log; exit 1; }
tail -2 gpurun_out/hot_tests.log
timeout -k 10 200 python tools/exp_variants.py 24 8 zipf walk uniform
