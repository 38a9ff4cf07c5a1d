set -e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/walk_prof -o walk -- python3 $GRAFT_REPO_ROOT/tools/exp_variants.py 24 6 walk > $GRAFT_REPO_ROOT/gpurun_out/walk_prof.log 2>&1
