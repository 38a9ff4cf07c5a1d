#!/bin/bash
# Tile-grouping check: its parity tests + the two-state parity/edge suites, then the C2 bench with the
# tile grouping and with the radix grouping (default) against the opt-in tile grouping (SG_GROUP_TILES=1), and a kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r02i}
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_ingest.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/grp_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/grp_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/grp_tests_$TAG.log
echo "== bench tile $(date +%T)"
SG_GROUP_TILES=1 timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/bench_tile_$TAG.json 2> gpurun_out/bench_tile_$TAG.err || { tail -30 gpurun_out/bench_tile_$TAG.err; exit 1; }
echo "== bench radix $(date +%T)"
timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/bench_radix_$TAG.json 2> gpurun_out/bench_radix_$TAG.err || { tail -30 gpurun_out/bench_radix_$TAG.err; exit 1; }
for k in tile radix; do python -c "
import json;d=json.loads(open('gpurun_out/bench_${k}_$TAG.json').read().strip().splitlines()[-1])
print('$k', '%.3e'%d['value'], d['ms_per_step'], d.get('stages_ms_per_step'), d.get('stages_ms_isolated'), d['roofline']['frac'])"; done
echo "== prof $(date +%T)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extra > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -3
