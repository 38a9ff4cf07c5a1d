#!/bin/bash
# the chain kernel's time per batch under ablation builds (siddhi-1_amd/lib_a{1,2,3}: no store / no walk / no load)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "" 1 2 3; do
  if [ -n "$v" ]; then export SG_HIP_LIBRARY=siddhi-1_amd/lib_a$v/libsiddhi_gpu.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/chn_abl$v -o chn -- python3 tools/exp_chain.py 6 > gpurun_out/chn_abl$v.log 2>&1 || exit 1
done
