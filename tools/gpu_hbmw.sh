# the wide HBM-pass window: two-state parity tests, then the C2 variants' stage times
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_hotkeys.py tests/test_gpu_grouping.py tests/test_gpu_pipeline.py tests/test_gpu_edges.py tests/test_gpu_snapshot.py tests/test_gpu_engine_reuse.py tests/test_gpu_projection.py > gpurun_out/hbmw_tests.log 2>&1 || { tail -30 gpurun_out/hbmw_tests.log; exit 1; }
tail -2 gpurun_out/hbmw_tests.log
echo "== new"; timeout -k 10 200 python tools/exp_variants.py 24 12 walk zipf uniform
