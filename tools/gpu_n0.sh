set -e
cd $GRAFT_REPO_ROOT
for n in 13 17 24; do echo "== N0=$n"; SG_HOT_N0=$n timeout -k 10 200 python tools/exp_variants.py 24 8 walk; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/zipf_prof -o zipf -- python3 $GRAFT_REPO_ROOT/tools/exp_variants.py 24 6 zipf > $GRAFT_REPO_ROOT/gpurun_out/zipf_prof.log 2>&1
