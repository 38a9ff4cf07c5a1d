# kernel traces of the C2 variants (Zipf keys, random-walk prices) on the current build: summaries only
set -e
cd /tmp && export TMPDIR=/tmp
for v in zipf walk; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/var_$v -o $v -- python3 $GRAFT_REPO_ROOT/tools/exp_variants.py 24 4 $v > /tmp/var_$v.log 2>&1
  python3 $GRAFT_REPO_ROOT/tools/rocpd_summary.py /tmp/var_$v/${v}_results.db > $GRAFT_REPO_ROOT/gpurun_out/c2_${v}_kernel_stats.txt 2>&1
done
