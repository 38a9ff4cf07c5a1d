set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_baseline_configs.py tests/test_gpu_ingest.py tests/test_gpu_general.py tests/test_gpu_purge.py tests/test_gpu_snapshot.py -x -v --timeout 300 --timeout-method thread -s > gpurun_out/t1.log 2>&1; rc=$?; tail -40 gpurun_out/t1.log; exit $rc
