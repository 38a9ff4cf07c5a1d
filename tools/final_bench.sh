# the round's bench line, then the same C2 leg under a kernel trace (per-kernel averages for the roofline check)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 800 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/bench_prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 16 --no-extra --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof.err
