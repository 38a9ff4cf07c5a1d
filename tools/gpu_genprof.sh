#!/bin/bash
# kernel-trace summary of the general-engine configs (C4, C3_min1) at bench sizes: where a step goes
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/genprof
for c in ${@:-C4 C3_min1}; do
  SG_EXP_STEPS=8 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/genprof/$c -o run -- \
      python3 $R/tools/exp_gen.py $c > $R/gpurun_out/genprof/$c.log 2>&1 || exit 1
  find $R/gpurun_out/genprof/$c -type f ! -name '*stats*' -delete
done
