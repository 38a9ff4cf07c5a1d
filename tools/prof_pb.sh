set -e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pb_prof -o pb -- $GRAFT_REPO_ROOT/tools/ubench/part_bench_e1 > $GRAFT_REPO_ROOT/gpurun_out/pb_prof.log 2>&1
